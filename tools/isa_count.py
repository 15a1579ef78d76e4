"""Static instruction mix of kernels in a hipcc --cuda-device-only -S listing.

  hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S -o k.s sng_kernels.hip
  python tools/isa_count.py k.s step_lean_kernelILi10ELb1ELb0 step_wide_kernelILi10ELi2ELb1ELb0ELb0
"""
import collections
import re
import sys

text = open(sys.argv[1]).read()
for name, body in re.findall(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end", text, flags=re.S | re.M):
    if not any(k in name for k in sys.argv[2:]):
        continue
    ins = [ln.split()[0] for ln in body.split("\n") if ln.startswith("\t") and ln.strip() and not ln.strip().startswith((".", ";"))]
    c = collections.Counter()
    for i in ins:
        c["valu"] += i.startswith("v_")
        c["f64"] += i.startswith("v_") and "f64" in i
        c["salu"] += i.startswith("s_") and not i.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_barrier"))
        c["waitcnt"] += i.startswith("s_waitcnt")
        c["vmem"] += i.startswith(("buffer_", "global_", "flat_"))
        c["lds"] += i.startswith("ds_")
        c["branch"] += i.startswith(("s_cbranch", "s_branch"))
    print(name[:70], len(ins), dict(c))
