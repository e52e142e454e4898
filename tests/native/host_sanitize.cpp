// Sanitizer driver for the host-only parts of libsgx.so (SURVEY §5 "Race detection /
// sanitizers": an ASan/UBSan build of the C-ABI CPU code).  Built by
// tests/test_host_sanitize.py together with sparkucx_amd/csrc/{sgx_index,sgx_plan,
// sgx_errors,sgx_bootstrap}.cpp under -fsanitize=address,undefined; every check failure or
// sanitizer report fails the test.  No GPU, no HIP headers.
#include <sys/wait.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sgx.h"
#include "../../sparkucx_amd/csrc/sgx_host.h"

static int failures = 0;
#define CHECK(c)                                                                            \
    do {                                                                                    \
        if (!(c)) {                                                                         \
            std::fprintf(stderr, "CHECK failed %s:%d: %s (%s)\n", __FILE__, __LINE__, #c,     \
                         sgx_last_error());                                                 \
            ++failures;                                                                     \
        }                                                                                   \
    } while (0)

static void placement_checks() {
    std::mt19937_64 rng(7);
    for (int P : {1, 2, 3, 8}) {
        for (int R : {1, 2, 7, 1024, 4099}) {
            std::vector<int64_t> L((size_t)P * R);
            for (auto &x : L) x = (int64_t)(rng() % 100 == 0 ? 100000 : rng() % 5000) * 16;
            std::vector<int32_t> b((size_t)P + 1);
            CHECK(sgx_balanced_ranges(L.data(), P, R, b.data()) == SGX_OK);
            CHECK(b[0] == 0 && b[(size_t)P] == R);
            for (int j = 0; j < P; ++j) CHECK(b[(size_t)j] <= b[(size_t)j + 1]);
            int64_t total = 0;
            for (int rank = 0; rank < P; ++rank) {
                std::vector<int64_t> sc(P), sd(P), rc(P), rd(P);
                int64_t n = 0;
                CHECK(sgx_plan_exchange_ranges(L.data(), P, R, rank, b.data(), 0, sc.data(), sd.data(), rc.data(),
                                               rd.data(), nullptr, &n) == SGX_OK);
                for (int j = 0; j < P; ++j) total += rc[j];
            }
            int64_t all = 0;
            for (int64_t x : L) all += x;
            CHECK(total == all);
            std::vector<int32_t> bad(b);
            if (P > 1) {
                bad[1] = R + 1;
                int64_t n = 0;
                std::vector<int64_t> sc(P), sd(P), rc(P), rd(P);
                CHECK(sgx_plan_exchange_ranges(L.data(), P, R, 0, bad.data(), 0, sc.data(), sd.data(), rc.data(),
                                               rd.data(), nullptr, &n) == SGX_ERR_INVALID);
            }
        }
    }
    std::vector<int64_t> zeros(12, 0);
    std::vector<int32_t> b(5), e(5);
    CHECK(sgx_balanced_ranges(zeros.data(), 4, 3, b.data()) == SGX_OK);
    CHECK(sgx_even_ranges(4, 3, e.data()) == SGX_OK);
    CHECK(b == e);
}

static void plan_checks() {
    placement_checks();
    std::mt19937_64 rng(42);
    for (int P : {1, 2, 3, 4, 8}) {
        for (int R : {1, 3, 200, 1024, 4099}) {
            std::vector<int64_t> L((size_t)P * R);
            for (auto &x : L) x = (int64_t)(rng() % 5000) * 16;
            std::vector<int64_t> total_recv(P, 0);
            for (int rank = 0; rank < P; ++rank) {
                std::vector<int64_t> sc(P), sd(P), rc(P), rd(P);
                int64_t n = 0;
                CHECK(sgx_plan_exchange(L.data(), P, R, rank, 4096, sc.data(), sd.data(), rc.data(), rd.data(),
                                        nullptr, &n) == SGX_OK);
                std::vector<int64_t> items((size_t)(n > 0 ? n : 1) * 3);
                int64_t cap = n;
                CHECK(sgx_plan_exchange(L.data(), P, R, rank, 4096, sc.data(), sd.data(), rc.data(), rd.data(),
                                        items.data(), &cap) == SGX_OK);
                CHECK(cap == n);
                int64_t mine = 0, sent = 0;
                for (int r = 0; r < R; ++r) mine += L[(size_t)rank * R + r];
                for (int j = 0; j < P; ++j) sent += sc[j];
                CHECK(sent == mine);
                int64_t recv = 0, copied = 0;
                for (int j = 0; j < P; ++j) recv += rc[j];
                for (int64_t i = 0; i < n; ++i) {
                    CHECK(items[3 * i + 2] > 0 && items[3 * i + 2] <= 4096);
                    CHECK(items[3 * i] >= 0 && items[3 * i] + items[3 * i + 2] <= recv);
                    CHECK(items[3 * i + 1] == copied);
                    copied += items[3 * i + 2];
                }
                CHECK(copied == recv);
                total_recv[rank] = recv;
                // too small a capacity is an error, never an overflow
                if (n > 1) {
                    int64_t small = n - 1;
                    CHECK(sgx_plan_exchange(L.data(), P, R, rank, 4096, sc.data(), sd.data(), rc.data(), rd.data(),
                                            items.data(), &small) == SGX_ERR_INVALID);
                }
            }
            int64_t all = 0, got = 0;
            for (auto x : L) all += x;
            for (auto x : total_recv) got += x;
            CHECK(all == got);
            for (int r = 0; r < R; ++r) {
                const int32_t o = sgx_reducer_owner(r, R, P);
                int32_t r0, r1;
                sgx::my_reducers(R, P, o, &r0, &r1);
                CHECK(o >= 0 && o < P && r0 <= r && r < r1);
            }
        }
    }
    int64_t z = 0, n = 0;
    CHECK(sgx_plan_exchange(nullptr, 1, 1, 0, 0, &z, &z, &z, &z, nullptr, &n) == SGX_ERR_INVALID);
    CHECK(sgx_reducer_owner(5, 4, 2) == -1);
}

static void index_checks(const std::string &dir) {
    const std::string idx = dir + "/shuffle_0_0_0.index", dat = dir + "/shuffle_0_0_0.data";
    std::vector<int64_t> lengths = {0, 16, 32, 0, 48};
    std::vector<uint8_t> data(96);
    for (size_t i = 0; i < data.size(); ++i) data[i] = (uint8_t)i;
    std::vector<int64_t> out(5, -1);
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, lengths.data(), data.data(), 96, out.data()) == SGX_OK);
    CHECK(out == lengths);
    std::vector<int64_t> chk(5, -1);
    CHECK(sgx_check_index_and_data(idx.c_str(), dat.c_str(), 5, chk.data()) == SGX_OK);
    CHECK(chk == lengths);
    int64_t off = -1, len = -1;
    CHECK(sgx_index_block_range(idx.c_str(), 2, 5, &off, &len) == SGX_OK);
    CHECK(off == 16 && len == 80);
    // a second attempt with other lengths: the first (valid) attempt wins
    std::vector<int64_t> other = {96, 0, 0, 0, 0};
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, other.data(), data.data(), 96, out.data()) == SGX_OK);
    CHECK(out == lengths);
    // mismatches are errors, not overflows
    CHECK(sgx_check_index_and_data(idx.c_str(), dat.c_str(), 4, chk.data()) == SGX_ERR_NOT_FOUND);
    CHECK(sgx_index_block_range(idx.c_str(), 0, 50, &off, &len) == SGX_ERR_IO);
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, other.data(), data.data(), 95, out.data()) ==
          SGX_ERR_INVALID);
    std::vector<int64_t> neg = {-16, 112, 0, 0, 0};
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, neg.data(), data.data(), 96, out.data()) ==
          SGX_ERR_INVALID);
    // a decreasing offset (a negative length) whose lengths still sum to the data size is
    // VALID for Spark (checkIndexAndDataFile only checks the count, off[0] == 0 and the sum,
    // IndexShuffleBlockResolver.scala:110-149): the existing attempt still wins
    FILE *f = std::fopen(idx.c_str(), "r+b");
    CHECK(f != nullptr);
    if (f) {
        uint8_t big[8] = {0x7f, 0, 0, 0, 0, 0, 0, 0};
        std::fseek(f, 16, SEEK_SET);
        std::fwrite(big, 1, 8, f);
        std::fclose(f);
    }
    CHECK(sgx_check_index_and_data(idx.c_str(), dat.c_str(), 5, chk.data()) == SGX_OK);
    CHECK(chk[1] > 0 && chk[2] < 0 && chk[0] + chk[1] + chk[2] + chk[3] + chk[4] == 96);
    std::vector<int64_t> won(chk);
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, other.data(), data.data(), 96, out.data()) == SGX_OK);
    CHECK(out == won);
    // a first offset != 0 is corrupt: replaced by the next attempt
    f = std::fopen(idx.c_str(), "r+b");
    if (f) {
        uint8_t one[8] = {0, 0, 0, 0, 0, 0, 0, 1};
        std::fwrite(one, 1, 8, f);
        std::fclose(f);
    }
    CHECK(sgx_check_index_and_data(idx.c_str(), dat.c_str(), 5, chk.data()) == SGX_ERR_NOT_FOUND);
    CHECK(sgx::commit_index_files(idx.c_str(), dat.c_str(), 5, other.data(), data.data(), 96, out.data()) == SGX_OK);
    CHECK(out == other);
    // concurrent attempts of one map (Utils.tempFileWith names + the executor-wide commit lock):
    // exactly one wins, every attempt reports the winner's lengths, the files hold the winner's
    // bytes, and no temp file is left behind
    const std::string idx2 = dir + "/shuffle_0_7_0.index", dat2 = dir + "/shuffle_0_7_0.data";
    const int T = 8;
    std::vector<std::vector<int64_t>> att((size_t)T), got((size_t)T, std::vector<int64_t>(5, -1));
    std::vector<std::vector<uint8_t>> bytes((size_t)T, std::vector<uint8_t>(96));
    std::vector<int> rcs((size_t)T, -100);
    for (int t = 0; t < T; ++t) {
        att[(size_t)t] = {(int64_t)(16 * (t % 6)), 0, 0, 0, (int64_t)(96 - 16 * (t % 6))};
        for (size_t i = 0; i < 96; ++i) bytes[(size_t)t][i] = (uint8_t)(t * 31 + i);
    }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            rcs[(size_t)t] = sgx::commit_index_files(idx2.c_str(), dat2.c_str(), 5, att[(size_t)t].data(),
                                                     bytes[(size_t)t].data(), 96, got[(size_t)t].data());
        });
    for (auto &x : th) x.join();
    std::vector<int64_t> fin(5, -1);
    CHECK(sgx_check_index_and_data(idx2.c_str(), dat2.c_str(), 5, fin.data()) == SGX_OK);
    for (int t = 0; t < T; ++t) {
        CHECK(rcs[(size_t)t] == SGX_OK);
        CHECK(got[(size_t)t] == fin);
    }
    int winners = 0;
    for (int t = 0; t < T; ++t) {
        if (att[(size_t)t] != fin) continue;
        FILE *d = std::fopen(dat2.c_str(), "rb");
        std::vector<uint8_t> on(96);
        const bool same = d && std::fread(on.data(), 1, 96, d) == 96 && on == bytes[(size_t)t];
        if (d) std::fclose(d);
        winners += same ? 1 : 0;
    }
    CHECK(winners == 1);
    const std::string ls = "ls -1 '" + dir + "' | grep -c 'shuffle_0_7_0\\.\\(index\\|data\\)\\.' > '" + dir +
                           "/tmpcount' || true";
    CHECK(std::system(ls.c_str()) == 0);
    FILE *cf = std::fopen((dir + "/tmpcount").c_str(), "r");
    int leftover = -1;
    if (cf) {
        if (std::fscanf(cf, "%d", &leftover) != 1) leftover = -1;
        std::fclose(cf);
    }
    CHECK(leftover == 0);
}

static void bootstrap_checks() {
    uint8_t id[128];
    for (int i = 0; i < 128; ++i) id[i] = (uint8_t)(i * 7 + 1);
    const int port = 20000 + (int)(getpid() % 20000);
    const int nranks = 4;
    std::vector<std::thread> joiners;
    std::vector<int> ok(nranks, 0);
    for (int r = 1; r < nranks; ++r)
        joiners.emplace_back([&, r] {
            uint8_t got[128];
            int32_t nr = 0;
            if (sgx_bootstrap_join("127.0.0.1", port, r, 20000, got, &nr) == SGX_OK && nr == nranks &&
                std::memcmp(got, id, 128) == 0)
                ok[(size_t)r] = 1;
        });
    CHECK(sgx_bootstrap_serve(port, nranks, id, 20000) == SGX_OK);
    for (auto &t : joiners) t.join();
    for (int r = 1; r < nranks; ++r) CHECK(ok[(size_t)r] == 1);
    uint8_t got[128];
    int32_t nr = 0;
    CHECK(sgx_bootstrap_join("127.0.0.1", port + 1, 1, 300, got, &nr) == SGX_ERR_TIMEOUT);
}

int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    plan_checks();
    index_checks(dir);
    bootstrap_checks();
    // the error message is thread-local
    std::thread t([] { sgx::fail_msg(SGX_ERR_IO, "from another thread"); });
    t.join();
    CHECK(std::strstr(sgx_last_error(), "another thread") == nullptr);
    std::printf("host sanitize: %d failures\n", failures);
    return failures ? 1 : 0;
}
