"""CPU checks of the integer identities the kernels rely on (restated in numpy):

* mod_u32 (sgx_kernels.hip): Granlund-Montgomery round-up multiplier, exact u mod R for
  every 32-bit u and 2 <= R < 2^31 with the parameters of mod_params (sgx_internal.h);
* KIND_HASH_POW2: Utils.nonNegativeMod(h, R) == h & (R - 1) for power-of-two R
  (reference: Spark Utils.nonNegativeMod, HashPartitioner.getPartition)."""
import numpy as np

M32 = (1 << 32) - 1


def mod_params(R):
    l = (R - 1).bit_length()
    return ((1 << 32) * ((1 << l) - R)) // R + 1, l - 1


def mod_u32(u, R):
    m, s = mod_params(R)
    u = u.astype(np.uint64)
    t = (np.uint64(m) * u) >> np.uint64(32)
    q = (t + ((u - t) >> np.uint64(1))) >> np.uint64(s)
    return (u - q * np.uint64(R)) & np.uint64(M32)


def test_magic_modulo_exact():
    rng = np.random.default_rng(7)
    edge = np.array([0, 1, 2, 3, 0x7FFFFFFF, 0x80000000, 0x80000001, M32 - 1, M32], dtype=np.uint64)
    divisors = list(range(2, 8193)) + [12345, 65535, 65536, 65537, 1 << 20, (1 << 31) - 1, 1 << 30]
    for R in divisors:
        m, _ = mod_params(R)
        assert 0 <= m <= M32
        u = np.concatenate([edge, rng.integers(0, 1 << 32, 512, dtype=np.uint64),
                            np.uint64(R) * rng.integers(0, (1 << 32) // R, 64, dtype=np.uint64) + np.uint64(R - 1)])
        assert np.array_equal(mod_u32(u, R), u % np.uint64(R)), R


def test_pow2_hash_identity():
    rng = np.random.default_rng(3)
    h = np.concatenate([rng.integers(-(1 << 31), 1 << 31, 4096), [-(1 << 31), -1, 0, 1, (1 << 31) - 1]])
    for R in [1 << b for b in range(0, 14)]:
        want = np.mod(h, R)  # Java nonNegativeMod: ((h % R) + R) % R == floor mod
        assert np.array_equal(h.astype(np.int64) & (R - 1), want)
