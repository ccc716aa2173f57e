// TEST HARNESS -- exhaustive host check of the walk kernels' closed-form
// sqrt / reciprocal / Markstein division (wost_device.h unit_direction) against
// the IEEE operations they replace. Built and run by tests/test_unit_direction.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"

static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static float bf(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

extern "C" int unit_dir_check(long* counts) {
    long bad_sqrt = 0, bad_rcp = 0, bad_div = 0, n_div = 0;
    bool seen[65] = {};
    for (int k = -64; k <= 64; ++k) {
        const float s2 = bf(0x3F800000u + (uint32_t)k);
        const int j = k >= 0 ? (k >> 1) : -((1 - k) >> 1);
        const float dn = bf(0x3F800000u + (uint32_t)j);
        const float y = bf(j >= 0 ? 0x3F800000u - 2u * (uint32_t)j : 0x3F800000u + (uint32_t)((1 - j) >> 1));
        volatile float vs2 = s2, one = 1.0f;
        if (fb(std::sqrt((float)vs2)) != fb(dn)) ++bad_sqrt;
        if (fb(one / dn) != fb(y)) ++bad_rcp;
        if (seen[j + 32]) continue;   // neighbouring k share dn: check each dn once
        seen[j + 32] = true;
        // every mantissa of a in [1, 2); the exponent scales out for |a| >= 2^-100
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            const float a = bf(0x3F800000u | m);
            const float q = a * y;
            const float got = std::fma(std::fma(-q, dn, a), y, q);
            volatile float va = a, vdn = dn;
            ++n_div;
            if (fb(got) != fb(va / vdn)) ++bad_div;
        }
    }
    counts[0] = bad_sqrt; counts[1] = bad_rcp; counts[2] = bad_div; counts[3] = n_div;
    // the header's own function, on a few directions (both paths)
    long bad_fn = 0;
    for (int i = 0; i < 200000; ++i) {
        const float th = (float)i * 3.14159265e-5f;
        float c = std::cos(th), s = std::sin(th);
        if (i % 1000 == 7) { c *= 3.0f; }   // off the unit circle: IEEE path
        float dn, dx, dy;
        wost::unit_direction(c, s, dn, dx, dy);
        volatile float vc = c, vs = s;
        const float en = std::sqrt(vc * vc + vs * vs);
        if (fb(dn) != fb(en) || fb(dx) != fb(vc / en) || fb(dy) != fb(vs / en)) ++bad_fn;
    }
    counts[4] = bad_fn;
    return 0;
}
