"""Generate the LZ4BlockOutputStream golden fixtures (lz4_*.npz) WITHOUT the oracle.

The frames are built from the system liblz4 (LZ4_compress_default, 1.9.x, the same library
generation lz4-java 1.7.1 bundles for Spark 3.0.1) and the `xxhash` Python module (XXH32), with
lz4-java's LZ4BlockOutputStream framing written out here: "LZ4Block" | method|level |
compressedLen | originalLen | checksum & 0x0FFFFFFF (LE32) | payload, RAW when compression does
not shrink the block, a 21-byte end mark per non-empty partition stream.  The inputs are Kryo
streams of (Long, Long) records (oracle-independent numpy framing below) and byte patterns.

Run in this container: python tests/golden/make_golden_lz4.py
"""
import ctypes
import os

import numpy as np
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))
LZ4 = ctypes.CDLL("liblz4.so.1")
LZ4.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
SEED = 0x9747B28C


def compress(block: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(block) + len(block) // 255 + 64)
    n = LZ4.LZ4_compress_default(block, out, len(block), len(out))
    assert n > 0
    return out.raw[:n]


def level(block_size: int) -> int:
    return max(0, (block_size - 1).bit_length() - 10)


def frame_stream(data: bytes, block_size: int) -> bytes:
    if not data:
        return b""
    lv = level(block_size)
    out = bytearray()
    for p in range(0, len(data), block_size):
        blk = data[p:p + block_size]
        c = compress(blk)
        raw = len(c) >= len(blk)
        pay = blk if raw else c
        out += b"LZ4Block" + bytes([(0x10 if raw else 0x20) | lv])
        out += len(pay).to_bytes(4, "little") + len(blk).to_bytes(4, "little")
        out += (xxhash.xxh32_intdigest(blk, SEED) & 0x0FFFFFFF).to_bytes(4, "little") + pay
    return bytes(out + b"LZ4Block" + bytes([0x10 | lv]) + bytes(12))


def kryo_pairs(keys, values) -> bytes:
    """writeClassAndObject(java.lang.Long) twice per record: 0x09 + zigzag varlong."""
    out = bytearray()
    for k, v in zip(keys, values):
        for x in (int(k), int(v)):
            z = ((x << 1) ^ (x >> 63)) & (2**64 - 1)
            out.append(0x09)
            for _ in range(8):
                if z < 0x80:
                    break
                out.append((z & 0x7F) | 0x80)
                z >>= 7
            out.append(z & 0xFF)
    return bytes(out)


def make(name, parts, block_size):
    stream = b"".join(parts)
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    np.cumsum([len(p) for p in parts], out=offs[1:])
    frames = [frame_stream(p, block_size) for p in parts]
    np.savez_compressed(os.path.join(HERE, name), stream=np.frombuffer(stream, np.uint8),
                        offsets=offs, block_size=np.int64(block_size),
                        framed=np.frombuffer(b"".join(frames), np.uint8),
                        lengths=np.array([len(f) for f in frames], dtype=np.int64))
    print(name, len(stream), "->", sum(len(f) for f in frames))


def main():
    rng = np.random.default_rng(20261016)
    # Kryo streams of hash-partitioned-like runs: small keys (compressible) and uniform keys
    parts = []
    for r in range(6):
        n = [0, 1, 700, 3000, 9000, 0][r]
        keys = rng.integers(-2**63, 2**63, n, dtype=np.int64) if r % 2 else rng.integers(0, 5000, n)
        parts.append(kryo_pairs(keys, np.arange(n)))
    make("lz4_kryo_R6.npz", parts, 32768)
    # byte patterns: incompressible (RAW), all-zero, exact block multiple, tiny (< 13 B), periodic
    parts = [rng.integers(0, 256, 40000, dtype=np.uint8).tobytes(), bytes(65536), b"abc",
             bytes(range(12)), (b"0123456789abcdef" * 5000)[:70001], b""]
    make("lz4_patterns_R6.npz", parts, 32768)
    # small block size (64 B: level 0) over a mixed stream
    parts = [kryo_pairs(rng.integers(0, 300, 200), np.arange(200)), rng.integers(0, 4, 999, dtype=np.uint8).tobytes()]
    make("lz4_bs64_R2.npz", parts, 64)


if __name__ == "__main__":
    main()
