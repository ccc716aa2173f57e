// TEST HARNESS -- AddressSanitizer / UndefinedBehaviorSanitizer run of libwost's
// host-side C++ (segment-tree builder wost_tree.cpp, sampler / Green's-norm tables
// wost_tables.cpp) and of the C oracle (oracle/wost_oracle.c), built by
// tests/test_sanitizers.py with -fsanitize=address,undefined -fno-sanitize-recover.
// Exercises ordinary, degenerate and extreme inputs; exits non-zero on a failed
// check (a sanitizer finding aborts the process by itself).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../../dcrmontecarlo_amd/csrc/wost_tables.h"
#include "../../dcrmontecarlo_amd/csrc/wost_tree.h"
#include "../../oracle/wost_oracle.h"

static int fails = 0;
#define CHECK(c) do { if (!(c)) { std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); ++fails; } } while (0)

static std::vector<float> polyline(std::mt19937& rng, int nv, int kind) {
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    std::vector<float> xy(2 * (size_t)nv);
    for (int i = 0; i < nv; ++i) {
        const float t = nv > 1 ? (float)i / (float)(nv - 1) : 0.f;
        switch (kind) {
        case 0: xy[2 * i] = 2.f * t - 1.f; xy[2 * i + 1] = 0.1f * std::sin(40.f * t); break;   // topography
        case 1: xy[2 * i] = std::cos(6.2831853f * t); xy[2 * i + 1] = std::sin(6.2831853f * t); break;   // circle
        case 2: xy[2 * i] = u(rng); xy[2 * i + 1] = u(rng); break;                              // random zig-zag
        default: xy[2 * i] = 0.5f; xy[2 * i + 1] = 0.5f; break;                                 // all one point
        }
    }
    return xy;
}

int main() {
    std::mt19937 rng(7);
    // --- segment trees: sizes around the leaf boundaries, degenerate polylines
    for (int kind = 0; kind < 4; ++kind)
        for (int nv : {2, 3, 9, 17, 64, 65, 1000, 10001})
            for (int leaf : {1, 4, 8, 13}) {
                const std::vector<float> xy = polyline(rng, nv, kind);
                wost::SegmentTreeHost t;
                const bool ok = wost::build_segment_tree(xy.data(), nv, leaf, &t);
                CHECK(ok);
                if (ok) {
                    CHECK(t.leaf >= 1);
                    CHECK(t.rec.size() % 16 == 0);
                    for (float v : t.rec) CHECK(!std::isnan(v));
                }
            }
    // --- tables
    std::vector<float> nodes(4097);
    wost::greens_sampler_nodes(nodes.data(), 4097);
    for (int i = 1; i < 4097; ++i) CHECK(nodes[i] >= nodes[i - 1]);
    wost::greens_sampler_nodes_jacobian(nodes.data(), 4097);
    for (int i = 1; i < 4097; ++i) CHECK(nodes[i] >= nodes[i - 1]);
    for (double sb : {1e-3, 0.5, 2.40625, 10.0, 999.0}) {
        wost::screened_sampler_nodes(nodes.data(), 4097, sb);
        for (int i = 1; i < 4097; ++i) CHECK(nodes[i] >= nodes[i - 1]);
        CHECK(std::isfinite(wost::screened_greens_norm(1.0, sb)));
        CHECK(std::isfinite(wost::screened_greens(0.5, 1.0, sb)));
    }
    std::vector<float> cells(4 * 256);
    wost::greens_norm_cells(cells.data(), 256, 256.0 / 12.0);
    for (float v : cells) CHECK(std::isfinite(v));
    std::vector<float> fix(9 * 33);
    wost::screened_fixed_nodes(fix.data(), 9, 33, std::log(41.0));
    for (int j = 0; j < 9; ++j)
        for (int i = 1; i < 33; ++i) CHECK(fix[j * 33 + i] >= fix[j * 33 + i - 1]);
    for (double s : {0.0, 1e-6, 1e-3, 1.0, 40.0, 300.0})
        for (double rho : {0.0, 1e-9, 0.5, 1.0 - 1e-12, 1.0}) {
            const double c = wost::screened_fixed_cdf(rho, s);
            CHECK(c >= 0.0 && c <= 1.0);
        }
    for (double x : {0.0, 1e-8, 1.0, 30.0, 700.0, 1e6}) CHECK(!std::isnan(wost::i0e_host(x)));
    for (double x : {1e-8, 1.0, 3.0, 50.0}) CHECK(std::isfinite(wost::k0_host(x)));
    // --- the oracle: queries on degenerate geometry, and small solves of each mode
    for (int kind = 0; kind < 4; ++kind) {
        const std::vector<float> xy = polyline(rng, 33, kind);
        std::vector<uint8_t> mask(31);
        std::vector<float> times(32);
        float out5[5];
        (void)orc_distance(xy.data(), 33, 0.1f, 0.2f);
        (void)orc_silhouette_distance(xy.data(), 33, 0.1f, 0.2f);
        orc_is_silhouette(xy.data(), 33, 0.1f, 0.2f, mask.data());
        orc_ray_intersection(xy.data(), 33, 0.1f, 0.2f, 0.6f, 0.8f, times.data());
        orc_intersect_polylines(xy.data(), 33, 0.1f, 0.2f, 0.6f, 0.8f, 0.3f, out5);
    }
    const float sq[] = {0, 0, 1, 0, 1, 1, 0, 1, 0, 0};
    const float top[] = {1, 1, 0, 1};
    orc_term tg[] = {{1.f, 0, 1}};
    orc_factor fg[] = {{1, {1.f, 0.f, 0, 0, 0, 0, 0, 0}}};   // monomial x
    orc_field g = {tg, 1, fg, 1, 0, nullptr, 0};
    orc_term ta[] = {{2.f, 0, 0}};
    orc_field a = {ta, 1, nullptr, 0, 0, nullptr, 0};
    std::vector<float> pts = {0.3f, 0.4f, 0.7f, 0.8f};
    std::vector<float> vals(2 * 64);
    std::vector<uint32_t> steps(2 * 64);
    for (int mode = 0; mode < 4; ++mode) {
        orc_problem pb = {sq, 5, mode & 1 ? top : nullptr, mode & 1 ? 2 : 0, &g, mode >= 2 ? &g : nullptr,
                          nullptr, mode == 3 ? &a : nullptr, 0.0};
        const int rc = orc_solve(&pb, pts.data(), 2, 64, 0, 128, 200, 1e-3f, 5, 1, vals.data(), steps.data());
        CHECK(rc == 0);
    }
    std::printf("sanitize_host: %d failed checks\n", fails);
    return fails ? 1 : 0;
}
