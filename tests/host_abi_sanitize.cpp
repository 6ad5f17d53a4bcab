// host_abi_sanitize.cpp -- runs the host-only parts of the C ABI under AddressSanitizer and
// UndefinedBehaviorSanitizer (sanitizers on the host code; GPU sanitizers are not
// available).  Built by tests/test_host_sanitizers.py with hipcc, -fsanitize on the host side only.
// Exercises: table builders, the max* bucket table, the rand() jump-ahead, the placement rule,
// and every entry point's argument checks (td_create fails before touching a device for bad
// parameters, and with TD_ENODEV / TD_EINVAL when no gfx950 device is visible).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "turbo_mi355x.h"

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                    \
        }                                                               \
    } while (0)

int main()
{
    CHECK(td_abi_version() == TD_ABI_VERSION);
    int ns[16], ls[16], no[32];
    CHECK(td_trellis_tables(ns, ls, no) == TD_OK);
    CHECK(td_trellis_tables(nullptr, nullptr, nullptr) == TD_OK);
    for (int K : {1, 40, 1024, 6144, 10000}) {
        std::vector<int> pi(K);
        CHECK(td_qpp_table(K, 3, 10, pi.data()) == TD_OK);
    }
    CHECK(td_qpp_table(0, 3, 10, ns) == TD_EINVAL);
    CHECK(td_qpp_table(10001, 3, 10, ns) == TD_EINVAL);
    CHECK(td_qpp_table(40, 3, 10, nullptr) == TD_EINVAL);
    CHECK(std::strlen(td_last_error()) > 0);
    // max* over a sweep of differences, both precisions, both algorithms
    for (int i = -20000; i <= 20000; ++i) {
        const double d = i * 0.00037;
        const double r = td_maxstar_host_f64(0.25, 0.25 + d, TD_ALGO_LOGMAP);
        CHECK(r >= std::fmax(0.25, 0.25 + d) && r <= std::fmax(0.25, 0.25 + d) + 0.69316);
        CHECK(td_maxstar_host_f64(0.25, 0.25 + d, TD_ALGO_MAXLOG) == std::fmax(0.25, 0.25 + d));
        const float rf = td_maxstar_host_f32(0.25f, 0.25f + (float)d, TD_ALGO_LOGMAP);
        CHECK(rf >= std::fmax(0.25f, 0.25f + (float)d));
        // the windowed schedule's one-read table (the bucket clamp at both ends included)
        const double q = td_maxstar_host_f64(0.25, 0.25 + d, TD_MAXSTAR_WINDOW_FAST);
        CHECK(q >= std::fmax(0.25, 0.25 + d) && q <= std::fmax(0.25, 0.25 + d) + 0.69316);
        CHECK(std::fabs(q - r) <= 0.05 + 1e-12);
        CHECK(td_maxstar_host_f32(0.25f, 0.25f + (float)d, TD_MAXSTAR_WINDOW_FAST) >= std::fmax(0.25f, 0.25f + (float)d));
    }
    uint32_t win[31];
    for (unsigned seed : {0u, 1u, 20261015u})
        for (unsigned long long draws : {0ull, 1ull, 6146ull, 123456789ull}) CHECK(td_rand_window(seed, draws, win) == TD_OK);
    CHECK(td_rand_window(1, 1, nullptr) == TD_EINVAL);
    const float slow[] = {2.39f, 2.38f, 2.38f, 2.38f, 2.40f, 2.38f, 2.49f};
    const float fast[] = {2.39f, 2.38f, 2.28f, 2.40f, 2.39f, 2.29f, 2.40f, 2.22f};
    CHECK(td_debug_placement_rule(slow, 7) == 0);
    CHECK(td_debug_placement_rule(fast, 3) == 0);   // fewer than TD_PLACEMENT_MIN (8) candidates
    CHECK(td_debug_placement_rule(fast, 8) == 1);
    CHECK(td_debug_placement_rule(nullptr, 3) == TD_EINVAL);
    // argument checks: no device is touched for bad parameters
    td_handle* h = nullptr;
    td_params p{40, 3, 10, 2, TD_ALGO_LOGMAP, TD_F64, 0};
    td_params bad = p;
    bad.K = 0;
    CHECK(td_create(&h, &bad) == TD_EINVAL && h == nullptr);
    bad = p;
    bad.iterations = 65;
    CHECK(td_create(&h, &bad) == TD_EINVAL);
    bad = p;
    bad.f1 = 2;   // not a permutation of K = 40
    CHECK(td_create(&h, &bad) == TD_EINVAL);
    bad = p;
    bad.algo = 7;
    CHECK(td_create(&h, &bad) == TD_EINVAL);
    CHECK(td_create(nullptr, &p) == TD_EINVAL);
    const int rc = td_create(&h, &p);   // no GPU here: TD_ENODEV (or TD_EHIP from the runtime)
    if (td_device_count() == 0) CHECK(rc == TD_ENODEV || rc == TD_EHIP);
    if (rc == TD_OK) td_destroy(h);
    CHECK(td_destroy(nullptr) == TD_OK);
    CHECK(td_reserve(nullptr, 8) == TD_EINVAL);
    CHECK(td_decode_device(nullptr, nullptr, 1, nullptr, 0, nullptr, nullptr) == TD_EINVAL);
    CHECK(td_decode_host(nullptr, nullptr, 1, nullptr, nullptr) == TD_EINVAL);
    CHECK(td_siso_host(nullptr, nullptr, nullptr, 1, nullptr, 43, 1) == TD_EINVAL);
    CHECK(td_set_window(nullptr, nullptr) == TD_EINVAL);
    CHECK(td_set_window_maxstar(nullptr, TD_WMAXSTAR_FAST) == TD_EINVAL);
    CHECK(td_debug_window_layout(nullptr, 0, 0, 0) == TD_EINVAL);
    CHECK(td_debug_workspace_bytes(nullptr, nullptr) == TD_EINVAL);
    CHECK(td_profile_enable(nullptr, 1) == TD_EINVAL);
    CHECK(td_synth_seed(nullptr, 1) == TD_EINVAL);
    CHECK(td_modulate(nullptr, 1, 1, nullptr, nullptr, nullptr) == TD_EINVAL);
    CHECK(td_demodulate(nullptr, nullptr, 1, 1, 1.0, nullptr, nullptr) == TD_EINVAL);
    std::printf("host ABI sanitizer run: %d failed checks\n", fails);
    return fails ? 1 : 0;
}
