"""The device's table-driven log2 (fastconsensus_amd/csrc/fc_log2.h, used by the Infomap
decisions) compiled for the host and held to <= 2.5 ulp of a long-double log2 on random
arguments over the range the map-equation terms take (counts / 2M: 2^-31 .. ~1, and a margin
above 1), including the neighbourhood of 1 from both sides (no cancellation there)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = r'''
#define __host__
#define __device__
#include "fc_log2.h"
#include <cmath>
#include <cstdio>
#include <random>
static const fc::Log2Entry T[49] = FC_LOG2_TABLE;
int main() {
    std::mt19937_64 g(7);
    double worst = 0;
    for (int i = 0; i < 400000; ++i) {
        double x;
        switch (i % 4) {
            case 0: x = (double)(g() % 2000000000ull + 1) * (1.0 / 2750726.0); break;
            case 1: x = std::ldexp(1.0 + (g() >> 11) * 0x1p-53, -(int)(g() % 32)); break;
            case 2: x = 1.0 + ((double)(g() >> 11) * 0x1p-53 - 0.5) * 0x1p-10; break;
            default: x = 1.0 + ((double)(g() >> 11) * 0x1p-53 - 0.5) * 0x1p-30; break;
        }
        const double a = fc::fc_log2(x, T);
        const long double ref = log2l((long double)x);
        const double r = (double)ref;
        const double ulp = std::fabs(std::nextafter(r, INFINITY) - r);
        const double u = ulp > 0 ? (double)(fabsl((long double)a - ref) / ulp) : (a == 0.0 ? 0.0 : 1e9);
        if (u > worst) worst = u;
    }
    printf("%.4f\n", worst);
}
'''


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_fc_log2_within_2_5_ulp(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-O2", "-I", os.path.join(ROOT, "fastconsensus_amd", "csrc"), str(src), "-o", str(exe)])
    worst = float(subprocess.check_output([str(exe)]).decode().strip())
    print("fc_log2 worst error %.3f ulp" % worst)
    assert worst <= 2.5
