// sgx_index.cpp — IndexShuffleBlockResolver's index + data layout
// (IndexShuffleBlockResolver.scala:56-262), host only (no HIP): index = (R+1) big-endian
// int64 offsets [0, L0, L0+L1, ...], data = the partition-contiguous bytes; commit through
// tmp files + rename, an existing valid attempt wins; the validation of checkIndexAndDataFile
// and the offset lookup of getBlockData.  Compiled into libsgx.so and, on its own, into the
// sanitizer build of the CPU suite.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sgx.h"
#include "sgx_host.h"

using sgx::fail_msg;

static bool read_file(const char *path, std::vector<uint8_t> &out) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    out.clear();
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + k);
    fclose(f);
    return true;
}

static int64_t file_size(const char *path) {
    struct stat st;
    if (stat(path, &st) != 0) return -1;
    return (int64_t)st.st_size;
}

static int64_t load_be64(const uint8_t *p) {
    uint64_t u = 0;
    for (int i = 0; i < 8; ++i) u = (u << 8) | p[i];
    return (int64_t)u;
}

// checkIndexAndDataFile (:110-149): lengths if index and data agree, else false.  The rules
// are exactly Spark's: (blocks + 1) longs, the first 0, and the data file as long as the sum of
// the lengths (offset differences, summed with Long wrap-around) -- a decreasing offset, i.e. a
// negative length, is NOT rejected on its own, as the reference does not reject it.
static bool check_index_and_data(const char *index_path, const char *data_path, int32_t blocks,
                                 std::vector<int64_t> &lengths) {
    const int64_t isz = file_size(index_path);
    if (isz != ((int64_t)blocks + 1) * 8) return false;
    std::vector<uint8_t> idx;
    if (!read_file(index_path, idx) || (int64_t)idx.size() != isz) return false;
    int64_t off = load_be64(idx.data());
    if (off != 0) return false;
    lengths.assign((size_t)blocks, 0);
    uint64_t sum = 0;  // Scala's lengths.sum wraps like uint64
    for (int32_t i = 0; i < blocks; ++i) {
        const int64_t nx = load_be64(idx.data() + 8 * (size_t)(i + 1));
        lengths[(size_t)i] = (int64_t)((uint64_t)nx - (uint64_t)off);
        sum += (uint64_t)lengths[(size_t)i];
        off = nx;
    }
    const int64_t dsz = file_size(data_path);
    return dsz >= 0 && (uint64_t)dsz == sum;
}

// Utils.tempFileWith (the reference's writeIndexFileAndCommit, :167): `<path>.<unique>`, so two
// attempts of one map -- each with its own map output object -- never share a temp file.
static std::string temp_file_with(const char *path) {
    static std::atomic<uint64_t> seq{0};
    const uint64_t t = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    char suffix[96];
    snprintf(suffix, sizeof suffix, ".%d.%llu.%llx", (int)getpid(), (unsigned long long)seq.fetch_add(1),
             (unsigned long long)(t * 0x9E3779B97F4A7C15ull));
    return std::string(path) + suffix;
}

// "There is only one IndexShuffleBlockResolver per executor, this synchronization make sure
// the following check and rename are atomic" (:170-171): one lock per process (= executor).
static std::mutex g_commit_mu;

extern "C" int sgx_check_index_and_data(const char *index_path, const char *data_path, int32_t blocks,
                                        int64_t *out_lengths) {
    if (!index_path || !data_path || blocks < 0) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    std::vector<int64_t> l;
    if (!check_index_and_data(index_path, data_path, blocks, l))
        return fail_msg(SGX_ERR_NOT_FOUND, "index %s and data %s do not match for %d blocks", index_path, data_path,
                        blocks);
    if (out_lengths && !l.empty()) std::memcpy(out_lengths, l.data(), sizeof(int64_t) * l.size());
    return SGX_OK;
}

extern "C" int sgx_index_block_range(const char *index_path, int32_t start, int32_t end, int64_t *off, int64_t *len) {
    if (!index_path || !off || !len || start < 0 || end < start) return fail_msg(SGX_ERR_INVALID, "bad arguments");
    FILE *f = fopen(index_path, "rb");
    if (!f) return fail_msg(SGX_ERR_IO, "cannot open index %s: %s", index_path, strerror(errno));
    uint8_t a[8], b[8];
    bool ok = fseek(f, (long)start * 8, SEEK_SET) == 0 && fread(a, 1, 8, f) == 8 &&
              fseek(f, (long)end * 8, SEEK_SET) == 0 && fread(b, 1, 8, f) == 8;
    // SPARK-22982 position check: after reading end's long we must sit at end*8+8.
    const bool pos_ok = ok && ftell(f) == (long)end * 8 + 8;
    fclose(f);
    if (!ok) return fail_msg(SGX_ERR_IO, "index %s too short for reduce range [%d, %d)", index_path, start, end);
    if (!pos_ok) return fail_msg(SGX_ERR_IO, "SPARK-22982: incorrect channel position after index file reads");
    *off = load_be64(a);
    *len = load_be64(b) - *off;
    return SGX_OK;
}

static int write_all(const char *path, const void *data, size_t n) {
    int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) return fail_msg(SGX_ERR_IO, "cannot create %s: %s", path, strerror(errno));
    const char *p = (const char *)data;
    while (n > 0) {
        ssize_t k = write(fd, p, n);
        if (k < 0) {
            if (errno == EINTR) continue;
            close(fd);
            return fail_msg(SGX_ERR_IO, "write %s: %s", path, strerror(errno));
        }
        p += k;
        n -= (size_t)k;
    }
    if (close(fd) != 0) return fail_msg(SGX_ERR_IO, "close %s: %s", path, strerror(errno));
    return SGX_OK;
}

// writeIndexFileAndCommit (:161-217) with the map output's bytes already on the host.
int sgx::commit_index_files(const char *index_path, const char *data_path, int32_t R, const int64_t *lengths,
                            const void *data, int64_t bytes, int64_t *out_lengths) {
    if (!index_path || !data_path || R < 1 || !lengths || bytes < 0 || (bytes > 0 && !data))
        return fail_msg(SGX_ERR_INVALID, "commit_index_files: bad arguments");
    int64_t sum = 0;
    for (int32_t i = 0; i < R; ++i) {
        if (lengths[i] < 0) return fail_msg(SGX_ERR_INVALID, "negative partition length at %d", i);
        sum += lengths[i];
    }
    if (sum != bytes) return fail_msg(SGX_ERR_INVALID, "lengths sum to %lld, data holds %lld", (long long)sum,
                                      (long long)bytes);
    const std::string data_tmp = temp_file_with(data_path);
    const std::string index_tmp = temp_file_with(index_path);
    // map output -> data tmp (dataTmp of writeIndexFileAndCommit, written before the lock)
    if (int rc0 = write_all(data_tmp.c_str(), data, (size_t)bytes)) {
        unlink(data_tmp.c_str());
        return rc0;
    }
    std::lock_guard<std::mutex> lk(g_commit_mu);
    std::vector<int64_t> existing;
    if (check_index_and_data(index_path, data_path, R, existing)) {
        // another attempt already committed: use its lengths, drop our data
        unlink(data_tmp.c_str());
        if (out_lengths) std::memcpy(out_lengths, existing.data(), sizeof(int64_t) * existing.size());
        return SGX_OK;
    }
    std::vector<uint8_t> idx((size_t)(R + 1) * 8);
    int64_t off = 0;
    for (int32_t i = 0; i <= R; ++i) {
        if (i > 0) off += lengths[i - 1];
        uint64_t u = (uint64_t)off;
        for (int b = 7; b >= 0; --b) {
            idx[(size_t)i * 8 + (size_t)b] = (uint8_t)(u & 0xFF);
            u >>= 8;
        }
    }
    int rc = write_all(index_tmp.c_str(), idx.data(), idx.size());
    if (rc) {
        unlink(index_tmp.c_str());
        unlink(data_tmp.c_str());
        return rc;
    }
    unlink(index_path);
    unlink(data_path);
    if (rename(index_tmp.c_str(), index_path) != 0) {
        unlink(index_tmp.c_str());
        unlink(data_tmp.c_str());
        return fail_msg(SGX_ERR_IO, "fail to rename file %s to %s", index_tmp.c_str(), index_path);
    }
    if (rename(data_tmp.c_str(), data_path) != 0) {
        unlink(data_tmp.c_str());
        return fail_msg(SGX_ERR_IO, "fail to rename file %s to %s", data_tmp.c_str(), data_path);
    }
    if (out_lengths) std::memcpy(out_lengths, lengths, sizeof(int64_t) * (size_t)R);
    return SGX_OK;
}
