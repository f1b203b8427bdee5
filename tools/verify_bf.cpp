// Host check of pt_math.h's branch-free Box-Muller forms against the branchy fdlibm logf /
// Cephes cosf restatements (logf_bf vs logf_pinned on [2^-32, 1] and at 0, cosf_bf vs
// cosf_pinned on [0, 2*pi]), every `stride`-th binary32 (stride 1 = exhaustive, ~40 s on 8
// threads).  Prints "<name> tested=<n> bad=<n>"; exit 1 on any mismatch.
#include "../opengl-path-tracing_amd/csrc/pt_math.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

int main(int argc, char** argv) {
    const unsigned stride = argc > 1 ? (unsigned)std::atoi(argv[1]) : 1u;
    int rc = 0;
    for (int which = 0; which < 2; which++) {
        const unsigned lo = which ? 0u : 0x2f800000u;               // 0 / 2^-32
        const unsigned hi = which ? 0x40c90fdcu : 0x3f800001u;      // RN(2*pi) / 1.0 inclusive
        std::atomic<unsigned long long> bad{0}, tested{0};
        auto worker = [&](unsigned t, unsigned nt) {
            unsigned long long nb = 0, n = 0;
            for (unsigned long long u = lo + (unsigned long long)t * stride; u < hi; u += (unsigned long long)nt * stride) {
                const float x = pt::bitsf((unsigned)u);
                const float a = which ? pt::cosf_bf(x) : pt::logf_bf(x);
                const float b = which ? pt::cosf_pinned(x) : pt::logf_pinned(x);
                n++;
                if (pt::fbits(a) != pt::fbits(b)) nb++;
            }
            bad += nb;
            tested += n;
        };
        std::vector<std::thread> th;
        const unsigned nt = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
        for (unsigned t = 0; t < nt; t++) th.emplace_back(worker, t, nt);
        for (auto& t : th) t.join();
        if (which == 0 && pt::fbits(pt::logf_bf(0.0f)) != pt::fbits(pt::logf_pinned(0.0f))) bad++;
        std::printf("%s tested=%llu bad=%llu\n", which ? "cosf_bf" : "logf_bf", tested.load(), bad.load());
        if (bad) rc = 1;
    }
    return rc;
}
