// TEST HARNESS -- host check that the walk kernels' split Philox draw
// (wost_device.h philox_walk / philox_draw) is bit for bit philox4x32_10 of the
// counter {k, 0, g_lo, g_hi}. Built and run by tests/test_philox_split.py.
#include <cstdint>

#include "../../dcrmontecarlo_amd/csrc/wost_device.h"

extern "C" long philox_split_check(long n) {
    long bad = 0;
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto next = [&s]() {   // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    for (long i = 0; i < n; ++i) {
        const uint64_t g = (i & 3) == 0 ? (uint64_t)i : next();
        const uint64_t key = (i & 7) == 1 ? 0ull : next();
        const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
        const wost::PhiloxWalk p = wost::philox_walk(g, k0, k1);
        for (uint32_t k : {0u, 1u, 2u, 77u, 999u, (uint32_t)next()}) {
            const wost::U4 a = wost::philox_draw(p, k, k0, k1);
            const wost::U4 b = wost::philox4x32_10(wost::U4{k, 0u, (uint32_t)g, (uint32_t)(g >> 32)}, k0, k1);
            bad += (a.x != b.x) || (a.y != b.y) || (a.z != b.z) || (a.w != b.w);
        }
    }
    return bad;
}
