// sgx_host.h — host-only helpers shared by every translation unit of libsgx.so, including
// the ones that never touch HIP (index files, exchange planning, bootstrap).  Those units
// are also compiled on their own with -fsanitize=address,undefined by the CPU test suite
// (tests/native/host_sanitize.cpp), so nothing here may include a HIP header.
#pragma once
#include <stdint.h>

namespace sgx {
// Sets the thread-local sgx_last_error() message and returns `code`.
int fail_msg(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// IndexShuffleBlockResolver.writeIndexFileAndCommit (IndexShuffleBlockResolver.scala:161-217)
// with the map output's `bytes` bytes on the host: data + index via tmp files and rename; an
// existing valid attempt wins and its lengths land in out_lengths (may be NULL).
int commit_index_files(const char *index_path, const char *data_path, int32_t R, const int64_t *lengths,
                       const void *data, int64_t bytes, int64_t *out_lengths);

// Reducer ownership floor(r * P / R) and its inverse: rank `rank` owns [*r0, *r1).
inline int32_t reducer_owner(int32_t r, int32_t R, int32_t P) { return (int32_t)(((int64_t)r * P) / R); }
inline void my_reducers(int32_t R, int32_t P, int32_t rank, int32_t *r0, int32_t *r1) {
    // owner(r) = floor(r*P/R) is monotone: [r0, r1) = { r : owner(r) == rank }
    const int32_t lo = (int32_t)(((int64_t)rank * R + P - 1) / P);
    const int32_t hi = (int32_t)(((int64_t)(rank + 1) * R + P - 1) / P);
    *r0 = lo < R ? lo : R;
    *r1 = hi < R ? hi : R;
}
}  // namespace sgx
