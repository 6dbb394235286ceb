// tests/cpp/libm_check.hip -- the device build of include/visionaray_hip/detail/vrh_libm.h against the
// host build of the same functions (which equal the host C library's sinf / cosf on every float input,
// tests/test_libm_sincosf.py) and against the host library itself.
//
//   libm_check <lo> <hi> <stride>
// evaluates vrh::libm::sinf / cosf on the GPU for the bit patterns lo, lo + stride, ... < hi, in
// chunks, and compares every result bit for bit (NaN results compare as NaN).  Prints one JSON line.
#include <hip/hip_runtime.h>

#include "visionaray_hip/detail/vrh_libm.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void eval(uint64_t lo, uint64_t stride, uint32_t n, float* s, float* c)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t u = uint32_t(lo + uint64_t(i) * stride);
    float x;
    memcpy(&x, &u, 4);
    s[i] = vrh::libm::sinf(x);
    c[i] = vrh::libm::cosf(x);
}

static bool same(float a, float b)
{
    if (std::isnan(a) || std::isnan(b)) return std::isnan(a) && std::isnan(b);
    return vrh::libm::asuint(a) == vrh::libm::asuint(b);
}

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)

int main(int argc, char** argv)
{
    if (argc < 4) { fprintf(stderr, "usage: libm_check lo hi stride\n"); return 2; }
    const uint64_t lo = strtoull(argv[1], nullptr, 0), hi = strtoull(argv[2], nullptr, 0), stride = strtoull(argv[3], nullptr, 0);
    if (stride == 0 || hi <= lo || hi > (1ull << 32)) { fprintf(stderr, "bad range\n"); return 2; }
    const uint64_t total = (hi - lo + stride - 1) / stride;
    const uint32_t chunk = 1u << 24;
    float *ds, *dc;
    CHECK(hipMalloc(&ds, chunk * sizeof(float)));
    CHECK(hipMalloc(&dc, chunk * sizeof(float)));
    std::vector<float> hs(chunk), hc(chunk);
    const unsigned nt = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    uint64_t bad_dev = 0, bad_lib = 0;
    long long first = -1;
    for (uint64_t k0 = 0; k0 < total; k0 += chunk)
    {
        const uint32_t n = uint32_t(std::min<uint64_t>(chunk, total - k0));
        const uint64_t base = lo + k0 * stride;
        hipLaunchKernelGGL(eval, dim3((n + 255) / 256), dim3(256), 0, 0, base, stride, n, ds, dc);
        CHECK(hipGetLastError());
        CHECK(hipMemcpy(hs.data(), ds, n * sizeof(float), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hc.data(), dc, n * sizeof(float), hipMemcpyDeviceToHost));
        std::vector<uint64_t> bd(nt, 0), bl(nt, 0);
        std::vector<long long> fd(nt, -1);
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                for (uint32_t i = t; i < n; i += nt)
                {
                    const uint32_t u = uint32_t(base + uint64_t(i) * stride);
                    float x;
                    memcpy(&x, &u, 4);
                    const float rs = vrh::libm::sinf(x), rc = vrh::libm::cosf(x);
                    if (!same(hs[i], rs) || !same(hc[i], rc)) { if (fd[t] < 0) fd[t] = u; ++bd[t]; }
                    if (!same(hs[i], ::sinf(x)) || !same(hc[i], ::cosf(x))) ++bl[t];
                }
            });
        for (auto& t : th) t.join();
        for (unsigned t = 0; t < nt; ++t)
        {
            bad_dev += bd[t];
            bad_lib += bl[t];
            if (first < 0 && fd[t] >= 0) first = fd[t];
        }
    }
    printf("{\"inputs\": %llu, \"lo\": %llu, \"hi\": %llu, \"stride\": %llu, \"device_vs_host_restatement\": %llu, "
           "\"device_vs_host_libm\": %llu, \"first_mismatch\": %lld, \"host_fma\": %d, \"host_avx2\": %d}\n",
           (unsigned long long)total, (unsigned long long)lo, (unsigned long long)hi, (unsigned long long)stride,
           (unsigned long long)bad_dev, (unsigned long long)bad_lib, first,
           __builtin_cpu_supports("fma") ? 1 : 0, __builtin_cpu_supports("avx2") ? 1 : 0);
    (void)hipFree(ds);
    (void)hipFree(dc);
    return bad_dev ? 1 : 0;
}
