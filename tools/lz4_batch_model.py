#!/usr/bin/env python3
"""Host model of the LZ4 compressor's multi-sequence batches (sgx_lz4.hip lz4_compress_batch),
lane for lane, checked against the oracle's LZ4_compress_default (oracle/lz4_oracle.c) on a
few block shapes.  A development check of the table-state argument (which entry each lane
sees, which lanes write at the batch end), not a test of the kernel: the GPU tests compare
the kernel itself with the oracle.   python tools/lz4_batch_model.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HASH_LOG, MINMATCH, LASTLIT, MFLIMIT = 13, 4, 5, 12


def skip_dist(m):
    if m == 0:
        return 0
    x = 62 + m
    q, r = x >> 6, x & 63
    return 1 + 32 * q * (q - 1) + q * (r + 1)


def compress(src):
    n = len(src)
    u32 = lambda i: int.from_bytes(src[i:i + 4], "little")
    hsh = lambda v: ((v * 2654435761) & 0xFFFFFFFF) >> (32 - HASH_LOG)
    table = [0] * (1 << HASH_LOG)
    out = bytearray()
    anchor = 0

    def emit(lit_from, lit_to, off, mlen):
        lit = lit_to - lit_from
        tok = (min(lit, 15) << 4) | min(mlen - MINMATCH, 15)
        out.append(tok)
        if lit >= 15:
            r = lit - 15
            while r >= 255:
                out.append(255)
                r -= 255
            out.append(r)
        out.extend(src[lit_from:lit_to])
        out.extend(off.to_bytes(2, "little"))
        if mlen - MINMATCH >= 15:
            r = mlen - MINMATCH - 15
            while r >= 255:
                out.append(255)
                r -= 255
            out.append(r)

    if n >= MFLIMIT + 1:
        lim, mlimit = n - MFLIMIT + 1, n - LASTLIT
        table[hsh(u32(0))] = 0
        start, it = 1, 0
        while True:  # batch
            pos = [start + skip_dist(it + j) for j in range(64)]
            valid = [p + max((it + j + 63) >> 6, 1) <= lim for j, p in enumerate(pos)]
            seq = [u32(min(p, n - 12)) for p in pos]
            h = [hsh(s) for s in seq]
            tcand = [table[x] for x in h]
            peers = [[i for i in range(64) if h[i] == h[j]] for j in range(64)]
            consec = it == 0
            W = set()
            lo = 0
            ended = False
            nxt = None
            while True:  # search in batch
                cand = []
                for j in range(64):
                    el = [i for i in peers[j] if i < j and (i in W or i >= lo)]
                    cand.append(pos[max(el)] if el else tcand[j])
                k = None
                kinv = 64
                for j in range(lo, 64):
                    if not valid[j]:
                        kinv = j
                        break
                    if u32(cand[j]) == seq[j]:
                        k = j
                        break
                kend = k + 1 if k is not None else kinv
                W |= set(range(lo, kend))
                if k is None:
                    if kinv < 64:
                        ended = True
                    else:
                        nxt = (start, it + 64) if lo == 0 else (start + lo, 64 - lo)
                    break
                ip, match = pos[k], cand[k]
                # catch up
                while ip > anchor and match > 0 and src[ip - 1] == src[match - 1]:
                    ip -= 1
                    match -= 1
                # LZ4_count from the hit's ip + 4 (the catch-up does not move the match end)
                d = cand[k] - pos[k]
                e = pos[k] + MINMATCH
                while e < mlimit and src[e] == src[e + d]:
                    e += 1
                aend = e
                lit_from = anchor
                cont = False
                first = True
                while True:  # _next_match
                    emit(lit_from if first else ip, ip, ip - match, aend - ip)
                    first = False
                    ip = aend
                    anchor = ip
                    if ip >= lim:
                        ended = True
                        break
                    a0 = ip - start
                    if consec and a0 < 64:
                        W.add(a0 - 2)
                        el = [i for i in peers[a0] if i < a0 and i in W]
                        m2 = pos[max(el)] if el else tcand[a0]
                        W.add(a0)
                        if u32(m2) != seq[a0]:
                            lo = a0 + 1
                            cont = lo < 64
                            if not cont:
                                nxt = (ip + 1, 0)
                            break
                        match = m2
                        e = ip + MINMATCH
                        while e < mlimit and src[e] == src[e + m2 - ip]:
                            e += 1
                        aend = e
                        continue
                    for j in W:  # the batch's insertions, then the serial test
                        if max(i for i in peers[j] if i in W) == j:
                            table[h[j]] = pos[j]
                    W = set()
                    table[hsh(u32(ip - 2))] = ip - 2
                    hh = hsh(u32(ip))
                    m2 = table[hh]
                    table[hh] = ip
                    if u32(m2) != u32(ip):
                        nxt = (ip + 1, 0)
                        break
                    match = m2
                    e = ip + MINMATCH
                    while e < mlimit and src[e] == src[e + m2 - ip]:
                        e += 1
                    aend = e
                if ended or not cont:
                    break
            for j in W:
                if max(i for i in peers[j] if i in W) == j:
                    table[h[j]] = pos[j]
            if ended:
                break
            start, it = nxt
    last = n - anchor
    out.append(min(last, 15) << 4)
    if last >= 15:
        r = last - 15
        while r >= 255:
            out.append(255)
            r -= 255
        out.append(r)
    out.extend(src[anchor:])
    return bytes(out)


def main():
    import oracle

    rng = np.random.default_rng(5)
    cases = {}
    recs = oracle.gen_uniform16(1 << 13, 7, value_base=3 << 32)
    st = oracle.kryo_serialize(recs).tobytes()
    cases["kryo_c1"] = st[:32768]
    cases["kryo_c1_tail"] = st[32768:32768 + 5000]
    cases["low_entropy"] = b"".join(int(i % 4096).to_bytes(8, "little") + int(i).to_bytes(8, "little")
                                    for i in range(2048))
    cases["random"] = rng.integers(0, 256, 32768, dtype=np.uint8).tobytes()
    cases["runs"] = bytes(rng.integers(0, 3, 32768, dtype=np.uint8))
    cases["periodic"] = (b"abcdefghij" * 4000)[:32768]
    cases["tiny"] = b"aaaaaaaaaaaaaaaaaaaa"
    bad = 0
    for name, blk in cases.items():
        want = oracle.lz4_compress_block(blk)
        got = compress(blk)
        ok = got == want
        bad += not ok
        print(f"{name}: {len(blk)} -> {len(want)} bytes, model {'==' if ok else '!='} oracle")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
