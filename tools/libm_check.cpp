// tools/libm_check.cpp -- exhaustive check of include/visionaray_hip/detail/vrh_libm.h against the
// host C library: every float input (2^32 of them, or the [lo, hi) range of bit patterns given),
// sinf and cosf, bit for bit (NaN results compare as NaN).  Prints the mismatch count per function
// and the CPU features that select glibc's variant (FMA + AVX2: __sinf_fma / __cosf_fma).
//   g++ -O2 -std=c++17 -ffp-contract=off -pthread -I include tools/libm_check.cpp -o libm_check
#include "visionaray_hip/detail/vrh_libm.h"

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static bool same(float a, float b)
{
    if (std::isnan(a) || std::isnan(b)) return std::isnan(a) && std::isnan(b);
    return vrh::libm::asuint(a) == vrh::libm::asuint(b);
}

int main(int argc, char** argv)
{
    const uint64_t lo = argc > 1 ? strtoull(argv[1], nullptr, 0) : 0ull;
    const uint64_t hi = argc > 2 ? strtoull(argv[2], nullptr, 0) : (1ull << 32);
    const unsigned nt = argc > 3 ? unsigned(atoi(argv[3])) : std::max(1u, std::thread::hardware_concurrency());
    std::atomic<uint64_t> bad_s{ 0 }, bad_c{ 0 }, first_s{ ~0ull }, first_c{ ~0ull };
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; ++k)
        th.emplace_back([&, k] {
            uint64_t bs = 0, bc = 0;
            for (uint64_t i = lo + k; i < hi; i += nt)
            {
                float x;
                const uint32_t u = uint32_t(i);
                std::memcpy(&x, &u, 4);
                if (!same(vrh::libm::sinf(x), ::sinf(x))) { if (!bs++) first_s = i; }
                if (!same(vrh::libm::cosf(x), ::cosf(x))) { if (!bc++) first_c = i; }
            }
            bad_s += bs;
            bad_c += bc;
        });
    for (auto& t : th) t.join();
    printf("{\"inputs\": %llu, \"lo\": %llu, \"hi\": %llu, \"sinf_mismatch\": %llu, \"cosf_mismatch\": %llu, "
           "\"first_sinf\": %lld, \"first_cosf\": %lld, \"fma\": %d, \"avx2\": %d}\n",
           (unsigned long long)(hi - lo), (unsigned long long)lo, (unsigned long long)hi,
           (unsigned long long)bad_s.load(), (unsigned long long)bad_c.load(),
           (long long)(bad_s ? first_s.load() : -1), (long long)(bad_c ? first_c.load() : -1),
           __builtin_cpu_supports("fma") ? 1 : 0, __builtin_cpu_supports("avx2") ? 1 : 0);
    return (bad_s || bad_c) ? 1 : 0;
}
