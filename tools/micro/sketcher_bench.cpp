// Per-call time of skq_sketcher_run from C++ (no Python in the loop): the drop-in's per-sequence
// path. usage: sketcher_bench [calls]
// build: g++ -O2 -std=c++17 -Iinclude tools/micro/sketcher_bench.cpp -o tools/micro/sketcher_bench \
//        -Lsketch-for-rna-seq_amd/lib -lskq -Wl,-rpath,$PWD/sketch-for-rna-seq_amd/lib
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "skq.h"

int main(int argc, char** argv) {
    const int calls = argc > 1 ? std::atoi(argv[1]) : 20000;
    skq_sketcher* h = nullptr;
    if (skq_sketcher_create(0, 4096, &h)) {
        std::fprintf(stderr, "create: %s\n", skq_last_error());
        return 1;
    }
    std::mt19937 rng(7);
    const char* acgt = "ACGT";
    std::vector<uint32_t> out(1 << 16);
    for (const int len : {0, 31, 150, 1500}) {
        std::string s(len, 'A');
        for (auto& c : s) c = acgt[rng() & 3];
        uint64_t cnt = 0, tot = 0;
        for (int i = 0; i < 200; ++i) skq_sketcher_run(h, s.data(), s.size(), 31, 214748367u, out.data(), out.size(), &cnt);
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < calls; ++i) {
            if (skq_sketcher_run(h, s.data(), s.size(), 31, 214748367u, out.data(), out.size(), &cnt)) {
                std::fprintf(stderr, "run: %s\n", skq_last_error());
                return 1;
            }
            tot += cnt;
        }
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / calls;
        std::printf("len %5d: %.2f us per call (%d calls, %.1f hashes per call)\n", len, us, calls, (double)tot / calls);
    }
    skq_sketcher_free(h);
    return 0;
}
