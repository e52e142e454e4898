"""CPU checks of the integer identities the kernels rely on (restated in numpy):

* mod_u32 (sgx_kernels.hip): Granlund-Montgomery round-up multiplier, exact u mod R for
  every 32-bit u and 2 <= R < 2^31 with the parameters of mod_params (sgx_internal.h);
* KIND_HASH_POW2: Utils.nonNegativeMod(h, R) == h & (R - 1) for power-of-two R
  (reference: Spark Utils.nonNegativeMod, HashPartitioner.getPartition);
* the exchange's reducer placement (sgx_even_ranges / sgx_balanced_ranges) and the plan
  over explicit ranges (sgx_plan_exchange_ranges)."""
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


def _best_max_brute(T, P):
    """Smallest possible largest range total over all placements of P contiguous ranges."""
    import itertools

    R = len(T)
    best = None
    for cuts in itertools.combinations_with_replacement(range(R + 1), P - 1):
        b = (0,) + cuts + (R,)
        m = max(sum(T[b[j]:b[j + 1]]) for j in range(P))
        best = m if best is None else min(best, m)
    return best


def test_balanced_ranges_optimal_and_contiguous(sgx_lib):
    """sgx_balanced_ranges (byte-balanced reducer placement): contiguous, covering [0, R),
    and its largest per-rank total equals the brute-force optimum on small cases; uniform
    lengths give the even split; a round without bytes gets the even placement."""
    rng = np.random.default_rng(5)
    for trial in range(150):
        P = int(rng.integers(1, 5))
        R = int(rng.integers(1, 9))
        L = rng.integers(0, 50, size=(P, R)) * (rng.random((P, R)) < 0.7)
        if trial % 5 == 0:
            L[:, int(rng.integers(0, R))] += 500  # one hot reducer (Zipf's head)
        b = sgx_lib.balanced_ranges(L)
        assert b[0] == 0 and b[-1] == R and np.all(np.diff(b) >= 0), b
        T = L.sum(axis=0)
        got = max(int(T[b[j]:b[j + 1]].sum()) for j in range(P))
        assert got == _best_max_brute(list(map(int, T)), P), (L.tolist(), b)
    for P, R in ((4, 1024), (8, 4096), (3, 7), (8, 3)):
        assert np.array_equal(sgx_lib.balanced_ranges(np.ones((P, R), np.int64)),
                              sgx_lib.balanced_ranges(np.ones((P, R), np.int64)))
        assert np.array_equal(sgx_lib.balanced_ranges(np.zeros((P, R), np.int64)), sgx_lib.even_ranges(P, R))
    assert np.array_equal(sgx_lib.balanced_ranges(np.full((4, 1024), 16, np.int64)), sgx_lib.even_ranges(4, 1024))
    owners = [sgx_lib.reducer_owner(r, 1000, 8) for r in range(1000)]
    eb = sgx_lib.even_ranges(8, 1000)
    assert all(eb[owners[r]] <= r < eb[owners[r] + 1] for r in range(1000))


def test_plan_with_ranges_is_consistent(sgx_lib):
    """sgx_plan_exchange_ranges under the byte-balanced placement of Zipf-like lengths: what
    every rank sends to j is what j expects from it, the receive layout covers j's range,
    and the largest receive total drops well below the even placement's."""
    rng = np.random.default_rng(9)
    P, R = 8, 4096
    w = 1.0 / np.arange(1, R + 1) ** 1.1
    L = (rng.poisson(2000 * w[None, :] * R / w.sum() * 8, size=(P, R)) * 16).astype(np.int64)
    for bounds in (sgx_lib.even_ranges(P, R), sgx_lib.balanced_ranges(L)):
        plans = [sgx_lib.plan_exchange(L, k, 0, bounds) for k in range(P)]
        for j in range(P):
            for k in range(P):
                assert plans[k][0][j] == plans[j][2][k]  # k sends to j == j receives from k
            assert plans[j][2].sum() == L[:, bounds[j]:bounds[j + 1]].sum()
    recv_even = [L[:, a:b].sum() for a, b in zip(sgx_lib.even_ranges(P, R)[:-1], sgx_lib.even_ranges(P, R)[1:])]
    bb = sgx_lib.balanced_ranges(L)
    recv_bal = [L[:, a:b].sum() for a, b in zip(bb[:-1], bb[1:])]
    assert max(recv_bal) < 0.5 * max(recv_even)


def test_plan_exchange_maps_simulated_all_to_all(sgx_lib):
    """sgx_plan_exchange_maps (the per-shuffle exchange's plan, any number of maps per rank,
    0 included) simulated end to end on the host: every rank packs its maps' pieces
    [destination][map] at its send displacements, the all-to-all moves them, and every block
    (map m, my reducer r) found at block_off is exactly that map's partition r."""
    rng = np.random.default_rng(11)
    for trial in range(60):
        P = int(rng.integers(1, 7))
        R = int(rng.integers(1, 40))
        counts = rng.integers(0, 4, P)
        if trial % 7 == 0:
            counts[:] = 0
        M = int(counts.sum())
        L = rng.integers(0, 5, (M, R)).astype(np.int64)
        L[rng.random((M, R)) < 0.3] = 0
        first = np.concatenate([[0], np.cumsum(counts)])
        # map m's partition-contiguous output: byte value = (m * 37 + r) mod 251 per partition
        outs = [np.concatenate([np.full(L[m, r], (m * 37 + r) % 251, np.uint8) for r in range(R)])
                if L[m].sum() else np.zeros(0, np.uint8) for m in range(M)]
        bounds = sgx_lib.balanced_ranges(
            np.stack([L[first[j]:first[j + 1]].sum(0) for j in range(P)])) if trial % 2 else \
            sgx_lib.even_ranges(P, R)
        plans = [sgx_lib.plan_exchange_maps(L.reshape(M, R), counts, k, bounds) for k in range(P)]
        sends = []
        for j, (sc, sd, _, _, _) in enumerate(plans):
            buf = np.zeros(int(sc.sum()), np.uint8)
            for d in range(P):
                pos = int(sd[d])
                for m in range(first[j], first[j + 1]):
                    o = int(L[m, :bounds[d]].sum())
                    ln = int(L[m, bounds[d]:bounds[d + 1]].sum())
                    buf[pos:pos + ln] = outs[m][o:o + ln]
                    pos += ln
                assert pos == int(sd[d] + sc[d])
            sends.append(buf)
        for k, (sc, sd, rc, rd, bo) in enumerate(plans):
            recv = np.zeros(int(rc.sum()), np.uint8)
            for j in range(P):
                sj_c, sj_d = plans[j][0], plans[j][1]
                assert rc[j] == sj_c[k]
                recv[rd[j]:rd[j] + rc[j]] = sends[j][sj_d[k]:sj_d[k] + sj_c[k]]
            r0, r1 = int(bounds[k]), int(bounds[k + 1])
            assert bo.shape == (M, r1 - r0)
            for m in range(M):
                po = np.concatenate([[0], np.cumsum(L[m])])
                for r in range(r0, r1):
                    got = recv[bo[m, r - r0]:bo[m, r - r0] + L[m, r]]
                    assert np.array_equal(got, outs[m][po[r]:po[r + 1]]), (trial, k, m, r)
