#!/usr/bin/env python3
"""Host check of the compact tables' placement (mph_place in skq_capi.hip) over bucket sizes and
loads: compiles the function from the source into a small harness with 4.24M random keys (cfg3's
key count below (double)0.05f's threshold) and reports success, time and pilot-array size.
usage: tools/mph_sweep.py [lambda:alpha ...]"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "sketch-for-rna-seq_amd", "csrc", "skq_capi.hip")).read()
i = src.index("bool mph_place(")
fn = src[i:src.index("\n}\n", i) + 3]
harness = r'''#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "skq_internal.h"
''' + fn + r'''
int main(int argc, char** argv) {
    const double lam = atof(argv[1]), alpha = atof(argv[2]);
    std::mt19937_64 g(1);
    std::vector<uint32_t> keys(4240000);
    for (auto& k : keys) k = (uint32_t)(g() % 214748367ull);
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const uint64_t m = keys.size(), nslots = (uint64_t)((double)m / alpha) + 1;
    const uint32_t nb = (uint32_t)std::max<uint64_t>(1, (uint64_t)(m / lam));
    std::vector<uint16_t> pil;
    std::vector<uint32_t> slot;
    const auto t0 = std::chrono::steady_clock::now();
    const bool ok = mph_place(keys, 0x5EED5EEDu, nslots, nb, pil, slot);
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("keys/bucket %4.1f load %.2f: %s in %.2f s, pilots %.0f KB, entries %.0f MB\n", lam, alpha,
                ok ? "placed" : "FAILED", dt, nb * 2 / 1024.0, nslots * 32 / 1048576.0);
}
'''
with tempfile.TemporaryDirectory() as d:
    c, exe = os.path.join(d, "h.cpp"), os.path.join(d, "h")
    open(c, "w").write(harness)
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                           "-I" + os.path.join(ROOT, "sketch-for-rna-seq_amd", "csrc"), c, "-o", exe])
    for arg in sys.argv[1:] or ["5:0.95", "8:0.9", "8:0.85", "10:0.85", "12:0.8", "16:0.8", "24:0.7"]:
        lam, alpha = arg.split(":")
        subprocess.call([exe, lam, alpha], timeout=300)
