// Writes tests/golden/philox_rocrand.json: Random123 known-answer vectors for
// Philox4x32-10 and draws of rocRAND's philox4x32_10_engine (host build of the
// rocRAND header) for the (seed, subsequence = walk id, draw = step) layout
// that libwost's kernel and the oracle use.
// Build & run: hipcc -O1 tools/rocrand_philox_kat.cpp -o /tmp/kat && /tmp/kat > tests/golden/philox_rocrand.json
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>

int main() {
    std::printf("{\n  \"random123\": [\n");
    // Random123 kat_vectors, philox4x32 10 rounds
    std::printf("    {\"ctr\": [0, 0, 0, 0], \"key\": [0, 0], \"out\": [\"6627e8d5\", \"e169c58d\", \"bc57ac4c\", \"9b00dbd8\"]},\n");
    std::printf("    {\"ctr\": [4294967295, 4294967295, 4294967295, 4294967295], \"key\": [4294967295, 4294967295], \"out\": [\"408f276d\", \"41c83b0e\", \"a20bc7c6\", \"6d5451fd\"]},\n");
    std::printf("    {\"ctr\": [608135816, 2242054355, 320440878, 57701188], \"key\": [2752067618, 698298832], \"out\": [\"d16cfe09\", \"94fdcceb\", \"5001e420\", \"24126ea1\"]}\n");
    std::printf("  ],\n  \"rocrand_stream\": [\n");
    const unsigned long long seeds[3] = {0ull, 0x123456789abcdefull, 31337ull};
    const unsigned long long wids[3] = {0ull, 4097ull, 5000000123ull};
    bool first = true;
    for (unsigned long long s : seeds)
        for (unsigned long long w : wids) {
            rocrand_device::philox4x32_10_engine e(s, w, 0);
            for (int k = 0; k < 4; ++k) {
                uint4 r = e.next4();
                std::printf("%s    {\"seed\": %llu, \"subsequence\": %llu, \"draw\": %d, \"out\": [\"%08x\", \"%08x\", \"%08x\", \"%08x\"]}",
                            first ? "" : ",\n", s, w, k, r.x, r.y, r.z, r.w);
                first = false;
            }
        }
    std::printf("\n  ]\n}\n");
    return 0;
}
