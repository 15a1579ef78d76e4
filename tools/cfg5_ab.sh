cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for l in libsng_prev libsng libsng_prev libsng; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2 > gpurun_out/c5_$l.log 2>&1 || exit $?
  echo "$l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_$l.log) $(grep -o '"reset_us": [0-9.]*' gpurun_out/c5_$l.log)"
done
