// Host check of the pinned Box-Muller log / cos (pt_math.h logf_pinned / cosf_pinned, the
// code the kernels run, compiled for the host) against the oracle's separate restatement
// (oracle/pt_oracle.cpp o_logf / o_cosf, linked in): the same bits for every `stride`-th
// binary32 of the hot-path domains, x in [2^-32, 1] and 0 for log, t in [0, 2 pi] for cos
// (stride 1 = exhaustive, ~20 s on 8 threads).  tools/verify_fastmath.hip closes the loop on
// the GPU (device bits = host bits).  Test infrastructure only (tests/test_exact_div.py).
//   g++ -O2 -std=c++17 -ffp-contract=off -march=x86-64-v3 -pthread tools/verify_bf.cpp oracle/pt_oracle.cpp
#include "../opengl-path-tracing_amd/csrc/pt_math.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

extern "C" float oracle_logf(float x);
extern "C" float oracle_cosf(float x);

int main(int argc, char** argv) {
    const unsigned stride = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1u;
    const unsigned nthr = std::max(1u, std::thread::hardware_concurrency());
    int rc = 0;
    for (int which = 0; which < 2; which++) {
        const unsigned lo = which ? 0u : 0x2f800000u, hi = which ? 0x40c90fdcu : 0x3f800000u;   // inclusive
        std::atomic<unsigned long long> tested{0}, bad{0};
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nthr; t++) {
            th.emplace_back([&, t]() {
                unsigned long long n = 0, b = 0;
                for (unsigned long long u = (unsigned long long)lo + (unsigned long long)t * stride; u <= hi;
                     u += (unsigned long long)nthr * stride) {
                    const float x = pt::bitsf((uint32_t)u);
                    const float a = which ? pt::cosf_pinned(x) : pt::logf_pinned(x);
                    const float c = which ? oracle_cosf(x) : oracle_logf(x);
                    n++;
                    if (pt::fbits(a) != pt::fbits(c)) b++;
                }
                tested += n;
                bad += b;
            });
        }
        for (auto& x : th) x.join();
        if (which == 0 && pt::fbits(pt::logf_pinned(0.0f)) != pt::fbits(oracle_logf(0.0f))) bad++;
        std::printf("%s tested=%llu bad=%llu\n", which ? "cosf_pinned" : "logf_pinned", tested.load(), bad.load());
        if (bad.load()) rc = 1;
    }
    return rc;
}
