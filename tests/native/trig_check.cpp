// TEST HARNESS -- host check of the walk kernels' direction cos/sin (wost_device.h
// sincos_rn) against the C library's double cos/sin rounded once to float32 (the
// correctly rounded values but for ~1e-8 of the angles). Built and run by
// tests/test_trig_rn.py: every angle (u01(v) * 2) * pi of :226 (all 2^24 draws) and
// n_half angles theta / 2 + phi of :227-228 for the given segment angles phi.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"

using namespace wost;

static uint32_t fb(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }

static void one(float t, long* c) {
    float s, co;
    sincos_rn(t, s, co);
    const float rs = (float)std::sin((double)t), rc = (float)std::cos((double)t);
    c[1] += fb(s) != fb(rs);
    c[2] += fb(co) != fb(rc);
    c[3] += fb(sinf(t)) != fb(rs);      // the C library's float functions, for the record
    c[4] += fb(cosf(t)) != fb(rc);
    ++c[0];
}

extern "C" int trig_check(const float* phi, int n_phi, long n_half, long* c) {
    for (int i = 0; i < 5; ++i) c[i] = 0;
    for (uint32_t v = 0; v < (1u << 24); ++v) one((u01(v << 8) * 2.0f) * kPiF, c);
    uint64_t st = 0x9E3779B97F4A7C15ull;
    for (long i = 0; i < n_half && n_phi > 0; ++i) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        const float th = (u01((uint32_t)(st >> 32)) * 2.0f) * kPiF;
        one(th / 2.0f + phi[(st >> 8) % (uint64_t)n_phi], c);
    }
    return 0;
}
