// Host-side cost of moving small buffers into / out of pinned host memory of
// each allocation kind the small-allreduce service could use (rdc_service.h),
// median microseconds per copy.  No kernel runs.
//   g++ -O2 -mavx2 -std=c++17 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ -o tools/mailbox_probe \
//       tools/mailbox_probe.cc -L/opt/rocm/lib -lamdhip64
#include <hip/hip_runtime_api.h>
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

template <typename F>
static double med(F f) {
    std::vector<double> t;
    for (int i = 0; i < 400; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        f();
        t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    struct K {
        const char* name;
        unsigned flags;
    } kinds[] = {{"uncached", hipHostMallocUncached | hipHostMallocMapped},
                 {"coherent", hipHostMallocCoherent | hipHostMallocMapped},
                 {"default", hipHostMallocDefault}};
    std::vector<char> src(1 << 16, 3), dst(1 << 16);
    std::string out = "{";
    for (auto& k : kinds) {
        char* box = nullptr;
        if (hipHostMalloc((void**)&box, 1 << 16, k.flags) != hipSuccess) {
            out += "\"" + std::string(k.name) + "\": \"alloc failed\", ";
            continue;
        }
        for (size_t sz : {(size_t)4096, (size_t)8192}) {
            auto add = [&](const char* what, double v) {
                char b[128];
                snprintf(b, sizeof b, "\"%s_%s_%zu\": %.3f, ", k.name, what, sz, v);
                out += b;
            };
            add("memcpy_in", med([&] { memcpy(box, src.data(), sz); asm volatile("" ::: "memory"); }));
            add("memcpy_out", med([&] { memcpy(dst.data(), box, sz); asm volatile("" ::: "memory"); }));
            add("u64_store_loop", med([&] {
                    volatile uint64_t* w = (volatile uint64_t*)box;
                    for (size_t j = 0; j < sz / 8; ++j) w[j] = j;
                }));
            add("u64_load_loop", med([&] {
                    volatile uint64_t* w = (volatile uint64_t*)box;
                    uint64_t s = 0;
                    for (size_t j = 0; j < sz / 8; ++j) s += w[j];
                    asm volatile("" ::"r"(s));
                }));
            add("nt_store_avx", med([&] {
                    for (size_t j = 0; j < sz; j += 32)
                        _mm256_stream_si256((__m256i*)(box + j), _mm256_loadu_si256((const __m256i*)(src.data() + j)));
                    _mm_sfence();
                }));
            add("nt_load_avx", med([&] {
                    for (size_t j = 0; j < sz; j += 32)
                        _mm256_storeu_si256((__m256i*)(dst.data() + j), _mm256_stream_load_si256((__m256i*)(box + j)));
                    asm volatile("" ::: "memory");
                }));
        }
        (void)hipHostFree(box);
    }
    out += "\"end\": 0}";
    printf("%s\n", out.c_str());
    return 0;
}
