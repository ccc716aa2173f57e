// Dumps the host sampler tables (wost_tables.cpp) for tests/test_tables_parallel.py: the
// threaded build must write the same bytes as the one-thread build (-DWOST_TABLES_SERIAL).
#include "wost_tables.h"
#include <cstdio>
#include <cstring>
#include <vector>
int main(int argc, char** argv) {
    std::vector<float> v(4097);
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "wb");
    wost::greens_sampler_nodes(v.data(), 4097); fwrite(v.data(), 4, v.size(), f);
    wost::greens_sampler_nodes_jacobian(v.data(), 4097); fwrite(v.data(), 4, v.size(), f);
    for (double sb : {0.01, 1.0, 10.0, 123.456, 1000.0}) { wost::screened_sampler_nodes(v.data(), 4097, sb); fwrite(v.data(), 4, v.size(), f); }
    std::vector<float> fx(129 * 257);
    wost::screened_fixed_nodes(fx.data(), 129, 257, 3.7135720667043078); fwrite(fx.data(), 4, fx.size(), f);
    fclose(f);
}
