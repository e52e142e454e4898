// sgx_range.cpp — RangePartitioner's bounds from the data (Spark 3.0.1 RangePartitioner:
// the rangeBounds initialiser, sketch and determineBounds; restated, see include/sgx.h and
// DESIGN.md §16): GPU reservoir sampling with Spark's seeds + determineBounds on the host.
#include "sgx_engine.h"

#include <algorithm>
#include <array>
#include <vector>
#include <cmath>
#include <cstring>

using namespace sgx;

namespace {

// scala.util.hashing.MurmurHash3 (Scala 2.12): bytesHash(data, seed), arraySeed = 0x3c074a61
inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint32_t mm3_mix_last(uint32_t h, uint32_t k) {
    k *= 0xcc9e2d51u;
    k = rotl32(k, 15);
    k *= 0x1b873593u;
    return h ^ k;
}
inline uint32_t mm3_mix(uint32_t h, uint32_t k) {
    h = mm3_mix_last(h, k);
    h = rotl32(h, 13);
    return h * 5u + 0xe6546b64u;
}
inline uint32_t mm3_avalanche(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
uint32_t mm3_bytes_hash(const uint8_t *d, int len, uint32_t seed) {
    uint32_t h = seed;
    int i = 0, rem = len;
    while (rem >= 4) {
        const uint32_t k = (uint32_t)d[i] | ((uint32_t)d[i + 1] << 8) | ((uint32_t)d[i + 2] << 16) |
                           ((uint32_t)d[i + 3] << 24);
        h = mm3_mix(h, k);
        i += 4;
        rem -= 4;
    }
    uint32_t k = 0;
    if (rem == 3) k ^= (uint32_t)d[i + 2] << 16;
    if (rem >= 2) k ^= (uint32_t)d[i + 1] << 8;
    if (rem >= 1) {
        k ^= (uint32_t)d[i];
        h = mm3_mix_last(h, k);
    }
    return mm3_avalanche(h ^ (uint32_t)len);
}

// org.apache.spark.util.random.XORShiftRandom.hashSeed: MurmurHash3 of the big-endian bytes
uint64_t xorshift_hash_seed(int64_t seed) {
    uint8_t b[8];
    for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((uint64_t)seed >> (56 - 8 * i));
    const uint32_t lo = mm3_bytes_hash(b, 8, 0x3c074a61u);
    const uint32_t hi = mm3_bytes_hash(b, 8, lo);
    return ((uint64_t)hi << 32) | (uint64_t)lo;
}

// scala.util.hashing.byteswap32
int32_t byteswap32(int32_t v) {
    uint32_t hc = (uint32_t)v * 0x9e3775cdu;
    hc = __builtin_bswap32(hc);
    return (int32_t)(hc * 0x9e3775cdu);
}

// java.util.Random (48-bit LCG): the seeds PartitionwiseSampledRDD.getPartitions gives each
// partition it samples (new Random(seed).nextLong() per partition, in partition order)
struct JavaRandom {
    uint64_t s;
    explicit JavaRandom(int64_t seed) : s(((uint64_t)seed ^ 0x5DEECE66Dull) & ((1ull << 48) - 1)) {}
    int32_t next(int bits) {
        s = (s * 0x5DEECE66Dull + 0xBull) & ((1ull << 48) - 1);
        return (int32_t)(uint32_t)(s >> (48 - bits));
    }
    int64_t next_long() {
        const int64_t hi = next(32);
        const int64_t lo = next(32);
        return (int64_t)((uint64_t)hi << 32) + lo;
    }
};

// XORShiftRandom on the host (setSeed = hashSeed) and java.util.Random.nextDouble over it
struct XorShift {
    uint64_t s;
    explicit XorShift(int64_t seed) : s(xorshift_hash_seed(seed)) {}
    uint64_t next(int bits) {
        s ^= s << 21;
        s ^= s >> 35;
        s ^= s << 4;
        return s & ((1ull << bits) - 1);
    }
    double next_double() { return (double)((next(26) << 27) + next(27)) * 0x1.0p-53; }
};

// GapSampling(f, rng, epsilon = 5e-11).advance: items to drop before the next kept one,
// (log(max(u, eps)) / log1p(-f)).toInt (a double past Int.MaxValue saturates, as in Scala)
int64_t gap_advance(XorShift &rng, double lnq) {
    const double u = std::max(rng.next_double(), 5e-11);
    const double g = std::log(u) / lnq;
    return g >= 2147483647.0 ? 2147483647 : (int64_t)g;
}

// column form of M^(2^t), t = 0..47, M = one XORShiftRandom step
std::vector<uint64_t> xorshift_jump_table() {
    auto step = [](uint64_t s) {
        s ^= s << 21;
        s ^= s >> 35;
        s ^= s << 4;
        return s;
    };
    auto apply = [](const uint64_t *cols, uint64_t v) {
        uint64_t r = 0;
        for (int b = 0; b < 64; ++b)
            if ((v >> b) & 1ull) r ^= cols[b];
        return r;
    };
    std::vector<uint64_t> t(48 * 64);
    for (int b = 0; b < 64; ++b) t[(size_t)b] = step(1ull << b);
    for (int lvl = 1; lvl < 48; ++lvl)
        for (int b = 0; b < 64; ++b)
            t[(size_t)lvl * 64 + (size_t)b] = apply(&t[(size_t)(lvl - 1) * 64], apply(&t[(size_t)(lvl - 1) * 64], 1ull << b));
    return t;
}

struct Cand {
    std::array<uint8_t, 10> k10;
    int64_t k64;
    float w;
};

}  // namespace

extern "C" int sgx_range_bounds(sgx_engine *e, const void *const *batches, const int64_t *nrecords, int32_t nbatches,
                                int32_t rb, int32_t mem_kind, int32_t num_partitions, int32_t rdd_id,
                                int32_t parent_rdd_id, int32_t sample_points_per_partition, void *out_bounds,
                                int32_t *out_nbounds) {
    sgx::TraceRange trace_("sgx_range_bounds");
    if (!e || !out_nbounds || (nbatches > 0 && (!batches || !nrecords))) return fail_msg(SGX_ERR_INVALID, "NULL argument");
    if (rb != 16 && rb != 100) return fail_msg(SGX_ERR_UNSUPPORTED, "range bounds need 16 B or 100 B records, not %d", rb);
    if (mem_kind != SGX_MEM_HOST && mem_kind != SGX_MEM_DEVICE) return fail_msg(SGX_ERR_INVALID, "unknown mem_kind");
    if (num_partitions < 1 || nbatches < 0 || sample_points_per_partition < 1)
        return fail_msg(SGX_ERR_INVALID, "bad partition / batch / sample counts");
    *out_nbounds = 0;
    if (num_partitions <= 1 || nbatches == 0) return SGX_OK;  // rangeBounds = Array.empty
    HIP_TRY(hipSetDevice(e->device));
    Ctx *c = e->ctx();
    if (!c) return SGX_ERR_HIP;
    hipStream_t st = c->st;
    const int kb = rb == 16 ? 8 : 10;
    // sampleSize capped at 1M; over-sample 3x per partition (RangePartitioner rangeBounds)
    const double sample_size = std::min((double)sample_points_per_partition * num_partitions, 1e6);
    const int64_t k = (int64_t)std::ceil(3.0 * sample_size / nbatches);
    {
        std::lock_guard<std::mutex> jl(e->jump_mu);
        if (e->jump_dev.p == nullptr) {
            const std::vector<uint64_t> jt = xorshift_jump_table();
            SGX_TRY(e->jump_dev.ensure(jt.size() * 8));
            HIP_TRY(hipMemcpy(e->jump_dev.p, jt.data(), jt.size() * 8, hipMemcpyHostToDevice));
        }
    }
    SGX_TRY(c->sample_winner.ensure((size_t)k * 8));
    SGX_TRY(c->sample_keys.ensure((size_t)k * (size_t)kb));
    std::vector<std::vector<uint8_t>> samples((size_t)nbatches);
    int64_t num_items = 0;
    for (int32_t i = 0; i < nbatches; ++i) {
        const int64_t n = nrecords[i];
        if (n < 0) return fail_msg(SGX_ERR_INVALID, "batch %d: %lld records", i, (long long)n);
        num_items += n;
        const int64_t kk = std::min(n, k);
        samples[(size_t)i].resize((size_t)(kk * kb));
        if (kk == 0) continue;
        const void *src = batches[i];
        if (mem_kind == SGX_MEM_HOST) {
            SGX_TRY(c->stage_input(src, (size_t)(n * rb), st, &src));
        }
        const int32_t seed = byteswap32((int32_t)((uint32_t)i ^ ((uint32_t)rdd_id << 16)));
        const uint64_t s0 = xorshift_hash_seed((int64_t)seed);  // Int seed widened to Long
        HIP_TRY(launch_reservoir(src, n, rb, kb, k, s0, (const uint64_t *)e->jump_dev.p,
                                 (long long *)c->sample_winner.p, c->sample_keys.p, st));
        HIP_TRY(hipMemcpyAsync(samples[(size_t)i].data(), c->sample_keys.p, (size_t)(kk * kb), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
    }
    if (num_items == 0) return SGX_OK;
    // candidates weighted by 1 / sampling probability; a partition holding much more than its
    // share is re-sampled instead (below)
    const double fraction = std::min(sample_size / (double)std::max<int64_t>(num_items, 1), 1.0);
    std::vector<Cand> cand;
    auto add = [&](const uint8_t *p, float w) {
        Cand c{};
        if (kb == 8) {
            int64_t v;
            std::memcpy(&v, p, 8);
            c.k64 = v;
        } else {
            std::memcpy(c.k10.data(), p, 10);
        }
        c.w = w;
        cand.push_back(c);
    };
    std::vector<int32_t> imbalanced;
    for (int32_t i = 0; i < nbatches; ++i) {
        const int64_t n = nrecords[i];
        const int64_t len = (int64_t)samples[(size_t)i].size() / kb;
        if (fraction * (double)n > (double)k) {
            imbalanced.push_back(i);
            continue;
        }
        if (len == 0) continue;
        const float w = (float)((double)n / (double)len);
        for (int64_t j = 0; j < len; ++j) add(samples[(size_t)i].data() + j * kb, w);
    }
    if (!imbalanced.empty()) {
        // new PartitionPruningRDD(rdd.map(_._1), imbalanced).sample(false, fraction,
        // byteswap32(-rdd.id - 1)): PartitionwiseSampledRDD seeds each kept partition with the
        // next nextLong() of java.util.Random(seed), in partition order, and runs a fresh
        // BernoulliSampler(fraction) on it -- XORShiftRandom(that seed); gap sampling when
        // fraction <= 0.4 (GapSampling: the first advance() at construction, then one per kept
        // item), else one nextDouble per item, kept iff <= fraction.  Weight (1 / fraction).toFloat.
        JavaRandom jr((int64_t)byteswap32((int32_t)(-(int64_t)parent_rdd_id - 1)));
        const float w = (float)(1.0 / fraction);
        for (int32_t i : imbalanced) {
            const int64_t n = nrecords[i];
            const int64_t pseed = jr.next_long();
            std::vector<int64_t> idx;
            if (fraction >= 1.0) {
                idx.resize((size_t)n);
                for (int64_t j = 0; j < n; ++j) idx[(size_t)j] = j;
            } else if (fraction <= 0.4) {
                XorShift rng(pseed);
                const double lnq = std::log1p(-fraction);
                for (int64_t pos = gap_advance(rng, lnq); pos < n; pos += 1 + gap_advance(rng, lnq))
                    idx.push_back(pos);
            } else {
                SGX_TRY(c->sample_winner.ensure((size_t)std::max<int64_t>(n, 8)));
                HIP_TRY(launch_bernoulli_flags(n, fraction, xorshift_hash_seed(pseed), (const uint64_t *)e->jump_dev.p,
                                               (uint8_t *)c->sample_winner.p, st));
                std::vector<uint8_t> flags((size_t)n);
                HIP_TRY(hipMemcpyAsync(flags.data(), c->sample_winner.p, (size_t)n, hipMemcpyDeviceToHost, st));
                HIP_TRY(hipStreamSynchronize(st));
                for (int64_t j = 0; j < n; ++j)
                    if (flags[(size_t)j]) idx.push_back(j);
            }
            if (idx.empty()) continue;
            const void *src = batches[i];
            if (mem_kind == SGX_MEM_HOST) {
                SGX_TRY(c->stage_input(src, (size_t)(n * rb), st, &src));
            }
            const int64_t m = (int64_t)idx.size();
            SGX_TRY(c->sample_winner.ensure((size_t)m * 8));
            SGX_TRY(c->sample_keys.ensure((size_t)m * (size_t)kb));
            HIP_TRY(hipMemcpyAsync(c->sample_winner.p, idx.data(), (size_t)m * 8, hipMemcpyHostToDevice, st));
            HIP_TRY(launch_gather_keys(src, rb, kb, (const int64_t *)c->sample_winner.p, m, c->sample_keys.p, st));
            std::vector<uint8_t> keys((size_t)(m * kb));
            HIP_TRY(hipMemcpyAsync(keys.data(), c->sample_keys.p, keys.size(), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            for (int64_t j = 0; j < m; ++j) add(keys.data() + j * kb, w);
        }
    }
    // determineBounds(candidates, min(partitions, candidates.size)): stable sort by key,
    // weights summed in sorted order, a bound each time the cumulative weight reaches the
    // next step, duplicates skipped
    auto lt = [kb](const Cand &a, const Cand &b) {
        return kb == 8 ? a.k64 < b.k64 : std::memcmp(a.k10.data(), b.k10.data(), 10) < 0;
    };
    std::stable_sort(cand.begin(), cand.end(), lt);
    const int32_t parts = (int32_t)std::min<int64_t>(num_partitions, (int64_t)cand.size());
    double sum_w = 0.0;
    for (const Cand &c : cand) sum_w += (double)c.w;
    const double step = sum_w / parts;
    double cum = 0.0, target = step;
    int32_t j = 0;
    const Cand *prev = nullptr;
    for (size_t i = 0; i < cand.size() && j < parts - 1; ++i) {
        cum += (double)cand[i].w;
        if (cum >= target) {
            if (!prev || lt(*prev, cand[i])) {
                if (out_bounds) {
                    if (kb == 8) std::memcpy((char *)out_bounds + (size_t)j * 8, &cand[i].k64, 8);
                    else std::memcpy((char *)out_bounds + (size_t)j * 10, cand[i].k10.data(), 10);
                }
                target += step;
                ++j;
                prev = &cand[i];
            }
        }
    }
    *out_nbounds = j;
    return SGX_OK;
}

