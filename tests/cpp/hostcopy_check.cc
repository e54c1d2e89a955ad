// rdc_amd::ParallelCopy (rdc_amd/csrc/rdc_copypool.h), the host path's
// pageable <-> pinned copy: every byte copied, none outside the range
// touched, for sizes around the part boundaries (the pool cuts a copy into
// up to 16 parts of 4 KiB multiples), misaligned ends, streaming stores on
// and off.
//   g++ -O2 -std=c++17 -pthread -I rdc_amd/csrc tests/cpp/hostcopy_check.cc
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "rdc_copypool.h"

int main() {
    const size_t kMin = (size_t)512 << 10;  // rdc_host.cpp kParallelMin
    rdc_amd::CopyPool pool(3);
    std::vector<size_t> sizes = {0, 1, 31, 32, 127, 128, 129, 4095, 4096, kMin - 1, kMin, kMin + 1,
                                 4 * (kMin / 2) + 3,  // floor(bytes / parts) a 4 KiB multiple, 3 left over
                                 16 * (kMin / 2) + 15, 16 * 4096 * 37 + 9, (size_t)8 << 20, ((size_t)8 << 20) + 4099,
                                 ((size_t)1 << 20) + 4099};
    std::mt19937_64 rng(12345);
    for (int i = 0; i < 40; ++i) sizes.push_back(kMin + rng() % ((size_t)12 << 20));
    for (int parts = 2; parts <= 16; ++parts)  // every part count with an exact 4 KiB floor and a remainder
        sizes.push_back((size_t)parts * (kMin / 2) + (size_t)parts - 1);
    const size_t guard = 64;
    long bad = 0, cases = 0;
    for (size_t S : sizes)
        for (int stream = 0; stream < 2; ++stream)
            for (size_t so : {(size_t)0, (size_t)3}) {
                const size_t dof = (so * 7 + (size_t)stream * 5) % 32;
                std::vector<char> src(S + guard + 32), dst(S + 2 * guard + 32);
                for (auto& c : src) c = (char)rng();
                memset(dst.data(), 0x5A, dst.size());
                char* d = dst.data() + guard + dof;
                rdc_amd::ParallelCopy(pool, d, src.data() + so, S, stream != 0, kMin);
                ++cases;
                bool ok = memcmp(d, src.data() + so, S) == 0;
                for (size_t g = 0; g < guard + dof; ++g) ok = ok && dst[g] == 0x5A;
                for (char* p = d + S; p < dst.data() + dst.size(); ++p) ok = ok && *p == 0x5A;
                if (!ok) {
                    ++bad;
                    printf("mismatch: bytes %zu stream %d src+%zu dst+%zu\n", S, stream, so, dof);
                }
            }
    printf("{\"cases\": %ld, \"bad\": %ld}\n", cases, bad);
    return bad ? 1 : 0;
}
