"""The bench's layout byte model (bench.step_kernel_bytes: what the step moves per env-step of a device-RNG
day) against the committed rocprofv3 PMC traffic of the same kernels (profiles/pmc_step_kernel.json,
FETCH_SIZE x 2 + WRITE_SIZE, separate passes): within 2 % at the headline (N = 10) and at config 5 (N = 50,
stochastic profiles), i.e. the step moves no bytes the model does not account for."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_layout_model_matches_pmc_traffic():
    import bench
    entries = json.load(open(os.path.join(ROOT, "profiles", "pmc_step_kernel.json")))
    seen = 0
    for e in entries:
        noise = e["chargers"] == 50   # config 5: stochastic profiles
        rd, wr = bench.step_kernel_bytes(e["chargers"], noise=noise)
        model = (rd + wr) * e["envs"]
        assert abs(e["bytes_per_launch"] / model - 1) < 0.02, (e["kernel"], e["bytes_per_launch"], model)
        seen += 1
    assert seen >= 2
