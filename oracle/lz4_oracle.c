/* CPU restatement of Spark's shuffle compression framing -- TEST INFRASTRUCTURE ONLY.
 *
 * Spark 3.0.1 `spark.shuffle.compress=true` (the default) with `spark.io.compression.codec=lz4`
 * (the default) wraps every partition stream of a map output separately
 * (ShufflePartitionPairsWriter.open -> SerializerManager.wrapStream -> LZ4CompressionCodec)
 * in lz4-java 1.7.1's LZ4BlockOutputStream(blockSize = 32 KiB, LZ4Factory.fastCompressor(),
 * XXHash32 streaming checksum seeded 0x9747b28c, syncFlush = false).  These are third-party
 * dependencies of the reference (spark-core_2.12:3.0.1, `pom.xml:90-95`; lz4-java 1.7.1 with
 * its bundled liblz4 1.9.2), not vendored in /root/reference; their published algorithms are
 * restated here.  The reference's own anchor is the data file the writer commits
 * (`NvkvShuffleMapOutputWriter.scala:172-246`, `IndexShuffleBlockResolver.scala:161-217`).
 *
 * Restated:
 *  * LZ4_compress_default for one block < 64 KiB + 11 B (liblz4 1.9.x lz4.c,
 *    LZ4_compress_generic with tableType byU16, noDict, acceleration 1): 13-bit hash of the
 *    4-byte little-endian sequence, a zero-initialised 8192-entry u16 position table,
 *    skip-accelerated search, backward catch-up, "test next position" after each match.
 *  * XXH32 (seed 0x9747b28c); lz4-java's asChecksum() masks the value with 0x0FFFFFFF.
 *  * LZ4BlockOutputStream frames: "LZ4Block" | token = method | level | compressedLen LE32 |
 *    originalLen LE32 | checksum LE32 | payload; method LZ4 (0x20) unless the compressed
 *    block is not smaller than the original, then RAW (0x10) with the original bytes;
 *    level = max(0, 32 - nlz(blockSize - 1) - 10) (5 for 32 KiB).  finish() appends a
 *    21-byte end mark (RAW | level, three zero words).  A partition that receives no
 *    record never opens its stream, so it has no bytes at all.
 *
 * Pinned in tests/test_lz4.py against the system liblz4 (LZ4_compress_default,
 * LZ4_decompress_safe) and the `xxhash` Python module.
 */
#include <stdint.h>
#include <string.h>

#define MINMATCH 4
#define LASTLITERALS 5
#define MFLIMIT 12
#define LZ4_MIN_LENGTH (MFLIMIT + 1)
#define SKIP_TRIGGER 6
#define HASH_LOG_U16 13 /* LZ4_HASHLOG (12) + 1 for the byU16 table */

static uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static uint32_t hash4(const uint8_t *p) {
    return (rd32(p) * 2654435761u) >> (MINMATCH * 8 - HASH_LOG_U16);
}

/* LZ4_compress_default(src, dst, n, LZ4_compressBound(n)) for 0 <= n < 65547.  Returns the
 * compressed size; dst must hold n + n/255 + 16 bytes. */
int orc_lz4_compress_block(const uint8_t *src, int n, uint8_t *dst) {
    uint16_t table[1 << HASH_LOG_U16];
    memset(table, 0, sizeof table);
    const uint8_t *ip = src, *anchor = src, *iend = src + n;
    const uint8_t *mflimit_plus_one = iend - MFLIMIT + 1;
    const uint8_t *matchlimit = iend - LASTLITERALS;
    uint8_t *op = dst;
    if (n < LZ4_MIN_LENGTH) goto last_literals;

    table[hash4(ip)] = 0;
    ip++;
    uint32_t fwd_h = hash4(ip);
    for (;;) {
        const uint8_t *match;
        uint8_t *token;
        {   /* find a match */
            const uint8_t *fwd = ip;
            int step = 1, search = 1 << SKIP_TRIGGER;
            for (;;) {
                uint32_t h = fwd_h;
                uint32_t cur = (uint32_t)(fwd - src);
                uint32_t midx = table[h];
                ip = fwd;
                fwd += step;
                step = search++ >> SKIP_TRIGGER;
                if (fwd > mflimit_plus_one) goto last_literals;
                match = src + midx;
                fwd_h = hash4(fwd);
                table[h] = (uint16_t)cur;
                if (rd32(match) == rd32(ip)) break;
            }
        }
        /* catch up */
        while (ip > anchor && match > src && ip[-1] == match[-1]) { ip--; match--; }
        {   /* literals */
            unsigned lit = (unsigned)(ip - anchor);
            token = op++;
            if (lit >= 15) {
                int len = (int)lit - 15;
                *token = 15 << 4;
                for (; len >= 255; len -= 255) *op++ = 255;
                *op++ = (uint8_t)len;
            } else {
                *token = (uint8_t)(lit << 4);
            }
            memcpy(op, anchor, lit);
            op += lit;
        }
    next_match:
        {
            uint32_t off = (uint32_t)(ip - match);
            *op++ = (uint8_t)off;
            *op++ = (uint8_t)(off >> 8);
            /* LZ4_count bounded by matchlimit */
            const uint8_t *a = ip + MINMATCH, *b = match + MINMATCH;
            while (a < matchlimit && *a == *b) { a++; b++; }
            unsigned mc = (unsigned)(a - (ip + MINMATCH));
            ip = a;
            if (mc >= 15) {
                *token += 15;
                mc -= 15;
                for (; mc >= 255; mc -= 255) *op++ = 255;
                *op++ = (uint8_t)mc;
            } else {
                *token += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimit_plus_one) break;
        table[hash4(ip - 2)] = (uint16_t)(ip - 2 - src);
        {   /* test next position */
            uint32_t h = hash4(ip);
            uint32_t cur = (uint32_t)(ip - src);
            match = src + table[h];
            table[h] = (uint16_t)cur;
            if (rd32(match) == rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fwd_h = hash4(++ip);
    }
last_literals:
    {
        size_t last = (size_t)(iend - anchor);
        if (last >= 15) {
            size_t acc = last - 15;
            *op++ = 15 << 4;
            for (; acc >= 255; acc -= 255) *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(last << 4);
        }
        memcpy(op, anchor, last);
        op += last;
    }
    return (int)(op - dst);
}

/* ------------------------------------------------------------------- XXH32 ------------ */
#define P1 2654435761u
#define P2 2246822519u
#define P3 3266489917u
#define P4 668265263u
#define P5 374761393u
static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t round32(uint32_t acc, uint32_t in) { return rotl(acc + in * P2, 13) * P1; }

uint32_t orc_xxh32(const uint8_t *p, int64_t len, uint32_t seed) {
    const uint8_t *end = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t *limit = end - 16;
        do {
            v1 = round32(v1, rd32(p)); v2 = round32(v2, rd32(p + 4));
            v3 = round32(v3, rd32(p + 8)); v4 = round32(v4, rd32(p + 12));
            p += 16;
        } while (p <= limit);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    while (p + 4 <= end) { h = rotl(h + rd32(p) * P3, 17) * P4; p += 4; }
    while (p < end) { h = rotl(h + (*p) * P5, 11) * P1; p++; }
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

/* ------------------------------------------------------ LZ4BlockOutputStream ----------- */
#define LZ4B_SEED 0x9747b28cu
#define LZ4B_HEADER 21

static int lz4b_level(int block_size) {
    int nlz = __builtin_clz((unsigned)(block_size - 1));
    int l = 32 - nlz - 10;
    return l > 0 ? l : 0;
}

static void wr32le(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* One partition stream of `len` bytes -> its LZ4BlockOutputStream bytes (0 bytes when len is
 * 0: the stream was never opened).  `dst` NULL only measures.  Returns the framed length. */
int64_t orc_lz4_frame_stream(const uint8_t *src, int64_t len, int block_size, uint8_t *dst) {
    static const uint8_t magic[8] = {'L', 'Z', '4', 'B', 'l', 'o', 'c', 'k'};
    if (len == 0) return 0;
    int level = lz4b_level(block_size);
    int64_t out = 0;
    uint8_t tmp[65536 + 65536 / 255 + 16];
    for (int64_t pos = 0; pos < len; pos += block_size) {
        int o = (int)((len - pos) < block_size ? (len - pos) : block_size);
        int c = orc_lz4_compress_block(src + pos, o, tmp);
        int raw = c >= o;
        int plen = raw ? o : c;
        if (dst) {
            uint8_t *h = dst + out;
            memcpy(h, magic, 8);
            h[8] = (uint8_t)((raw ? 0x10 : 0x20) | level);
            wr32le(h + 9, (uint32_t)plen);
            wr32le(h + 13, (uint32_t)o);
            wr32le(h + 17, orc_xxh32(src + pos, o, LZ4B_SEED) & 0x0FFFFFFFu);
            memcpy(h + LZ4B_HEADER, raw ? src + pos : tmp, (size_t)plen);
        }
        out += LZ4B_HEADER + plen;
    }
    if (dst) {
        uint8_t *h = dst + out;
        memcpy(h, magic, 8);
        h[8] = (uint8_t)(0x10 | level);
        memset(h + 9, 0, 12);
    }
    return out + LZ4B_HEADER;
}

/* A map output's partition streams (byte offsets offs[0..R]) framed one after the other.
 * Writes the framed lengths to out_lengths[R]; dst NULL only measures.  Returns the total. */
int64_t orc_lz4_frame_partitions(const uint8_t *src, const int64_t *offs, int32_t R, int block_size,
                                 uint8_t *dst, int64_t *out_lengths) {
    int64_t total = 0;
    for (int32_t r = 0; r < R; r++) {
        int64_t l = orc_lz4_frame_stream(src + offs[r], offs[r + 1] - offs[r], block_size,
                                         dst ? dst + total : NULL);
        out_lengths[r] = l;
        total += l;
    }
    return total;
}
