"""tools/trace_steady.py on a synthetic rocprofv3 kernel trace (CPU): writes are split at their
sample kernel, the warm-up writes are left out of the timed mean, and kernels launched after the
last write (not part of a regular write) do not count toward it."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, writes, tail):
    t = 1_000_000
    rows = []

    def add(name, us):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": str(t), "End_Timestamp": str(t + int(us * 1000))})
        t += int(us * 1000) + 500

    add("void sgx::k_gen_uniform16(unsigned long*, long)", 900.0)  # the input generator: left out
    for k4 in writes:
        add("void sgx::k_pad_sample<0, 16>(char const*, long, int)", 30.0)
        add("sgx::k_pad_caps(unsigned int const*, int, double, double)", 6.0)
        add("void sgx::k_scatter16_wc<100, 8, 8, 16, false, 1>(HIP_vector_type<unsigned int, 4u> const*)", k4)
        add("void sgx::k_scan<false>(unsigned int const*, unsigned int*, long, unsigned long*)", 24.0)
    for name, us in tail:  # launched after the last write
        add(name, us)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def test_timed_writes_exclude_warmup_and_trailing_kernels(tmp_path):
    path = str(tmp_path / "run_kernel_trace.csv")
    writes = [1900.0, 1850.0, 1800.0] + [1650.0] * 5
    _trace(path, writes, tail=[("void sgx::k_gather_frags(long const*, long)", 5000.0)])
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_steady.py"), path, "--warmup", "3"],
                         check=True, capture_output=True, text=True).stdout
    res = json.loads(out.strip().splitlines()[-1])
    assert res["writes"] == 8
    assert res["k4_us_per_write"] == writes
    per_write = [k4 + 30.0 + 6.0 + 24.0 for k4 in writes]
    assert res["map_side_us_per_write"] == [round(x, 1) for x in per_write]
    assert abs(res["map_side_us_timed_mean"] - (1650.0 + 60.0)) < 0.05
    assert abs(res["k4_us_timed_mean"] - 1650.0) < 0.05
    # 8.59 GB per write at 1.71 ms: 0.628 of 8 TB/s
    assert abs(res["map_side_frac_timed"] - 8.589934592e9 / 1710e-6 / 8e12) < 1e-3
