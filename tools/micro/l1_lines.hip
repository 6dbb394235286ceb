// Microbenchmark: cost of one wave-level global_load_dwordx4 by the number of distinct 64-B records
// its 64 lanes touch (1, 16 or 64), data resident in L2 (8 MB table).  Each lane chases a chain of
// dependent indices so the loop is load-bound; reports loads per microsecond per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <cstdlib>

__global__ __launch_bounds__(64) void chase(const float4* __restrict__ tab, uint32_t mask, int mode, int iters, float* out)
{
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t idx = (blockIdx.x * 2654435761u) & mask;
    float acc = 0.0f;
    for (int i = 0; i < iters; ++i)
    {
        uint32_t rec;
        if (mode == 0) rec = idx;                                       // 1 record per wave
        else if (mode == 1) rec = (idx + (lane >> 2) * 977u) & mask;    // 16 records (4 lanes each)
        else rec = (idx + lane * 977u) & mask;                          // 64 records
        // lane reads quarter (lane & 3) of its record in modes 0/1 (a cooperative 64-B fetch) or
        // quarter 0 in mode 2 (one 16-B piece of a per-lane record)
        const uint32_t q = mode == 2 ? 0u : (lane & 3u);
        const float4 v = tab[4u * rec + q];
        acc += v.x + v.y + v.z + v.w;
        idx = (idx * 1103515245u + 12345u + ((uint32_t)__builtin_amdgcn_readfirstlane((int)__float_as_uint(v.x)) & 1u)) & mask;
    }
    if (acc == 12345.0f) out[0] = acc;
}

int main(int argc, char** argv)
{
    const uint32_t nrec = argc > 1 ? (1u << atoi(argv[1])) : (1u << 17);   // default 128K records x 64 B = 8 MB
    std::vector<float> h(nrec * 16);
    std::mt19937 g(1);
    for (auto& x : h) x = float(g() & 0xFFFF) * 1e-3f;
    float4* d; float* o;
    hipMalloc(&d, h.size() * 4); hipMalloc(&o, 4);
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 4096, blocks = cus * 24;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int mode = 0; mode < 3; ++mode)
    {
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, nrec - 1, mode, iters, o);
        hipEventRecord(a);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, nrec - 1, mode, iters, o);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms = 0; hipEventElapsedTime(&ms, a, b);
        double loads = double(blocks) * iters;   // wave-level load instructions
        printf("table %u KB mode %d (%s): %.3f ms, %.2f wave-loads/us/CU, %.1f GB/s of lane data\n", nrec / 16, mode,
               mode == 0 ? "1 record/wave" : mode == 1 ? "16 records, 4 lanes each" : "64 records",
               ms, loads / (ms * 1e3) / cus, loads * 1024 / (ms * 1e-3) / 1e9);
    }
    return 0;
}
