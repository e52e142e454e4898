#!/usr/bin/env python3
"""Per-phase cycle split of the 8x16 hash scatter (diagnostic DIAG=6 build of K4: stamped
with s_memtime by wave 0 of every workgroup; the stamps serialise a little, so read the
SHARES, not the absolute time)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["SGX_SCATTER_DIAG"] = "6"
import sparkucx_amd as sgx  # noqa: E402

n, R = 1 << 28, int(sys.argv[1]) if len(sys.argv) > 1 else 1024
e = sgx.ShuffleEngine(0)
buf = e.alloc(n * 16)
e.gen_uniform16(buf, n, 0x5EEDC0DE)
e.register_shuffle(1, R)
fn = sgx.lib().sgx_diag_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = (ctypes.c_ulonglong * 8)()
e.write_map(1, 0, buf, n, 16)
e.sync()
fn(out, 1)
e.stats_reset()
for _ in range(3):
    e.write_map(1, 0, buf, n, 16)
e.sync()
fn(out, 1)
st = e.stats()
names = ["load+pid", "barrier after load", "rank (wave0)", "barrier after rank", "merge+scan",
         "rank..stage total", "drain issue", "barrier+cursor"]
v = list(out)
stage = v[5] - v[2] - v[3] - v[4]
tot = v[0] + v[1] + v[5] + v[6] + v[7]
print(f"R={R} scatter {st.ms['scatter'] / 3:.3f} ms/launch (stamped build)")
for nm, x in zip(names, v):
    print(f"  {nm:22s} {x / tot * 100:6.1f} %")
print(f"  {'stage (derived)':22s} {stage / tot * 100:6.1f} %")
