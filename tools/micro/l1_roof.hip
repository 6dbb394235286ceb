// tools/micro/l1_roof.hip -- the roof of the vector-memory path for the traversal kernel's access
// shape: dependent 64-B record gathers, one chain per lane (vrh_device.h ray_step: a node-pair
// record is 4 loads of 16 B from one 64-B-aligned record; the next record depends on the data).
//
// Every lane chases its own chain of random records in a table of `MB` megabytes.  The modes vary
// how many DISTINCT cache lines one wave-level load instruction touches, with the same 16 B per
// lane and the same dependent-chain structure:
//   0 per-lane   : 64 lanes -> 64 records (the kernel's shape for incoherent rays)
//   1 pair       : lanes 2k, 2k+1 share a record, different 16-B quarters -> 32 lines
//   2 quad       : 4 lanes share a record, each its own quarter -> 16 lines
//   3 quad-bcast : 4 lanes share a record and read the same quarter -> 16 lines, 1/4 the bytes
//   4 wave       : all 64 lanes read one record (quarter = lane & 3) -> 1 line
//   5 coalesced  : lane i reads 16 B at 16 i of a 1-KB block -> 8 x 128-B lines (granularity probe)
// Run it under rocprofv3 --pmc (TCP_TOTAL_CACHE_ACCESSES_sum, TD_TD_BUSY_sum, TA_TA_BUSY_sum,
// GRBM_GUI_ACTIVE, SQ_INSTS_VMEM_RD) to get L1 accesses per instruction and per CU-cycle for each
// shape; tools/l1_roof.py turns the two outputs into the roof that bench.py prices the kernel with.
//
//     l1_roof [MB=16] [waves_per_cu=20] [iters=2048]     prints one JSON line per mode
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

__global__ __launch_bounds__(256) void chase(const float4* __restrict__ tab, uint32_t nrec, int mode, int iters,
                                             float* out)
{
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t link = (gid * 2654435761u) % nrec;
    float acc = 0.0f;
    for (int i = 0; i < iters; ++i)
    {
        // the record this lane loads and the 16-B quarters it reads
        uint32_t rec = link, q0 = 0, q1 = 1, q2 = 2, q3 = 3;
        if (mode == 1) { rec = __shfl(link, lane & ~1u); q0 = q1 = q2 = q3 = (lane & 1u) * 2u; q1 += 1u; q3 += 1u; }
        else if (mode == 2 || mode == 3) { rec = __shfl(link, lane & ~3u); q0 = q1 = q2 = q3 = mode == 2 ? (lane & 3u) : 0u; }
        else if (mode == 4) { rec = __shfl(link, 0); q0 = q1 = q2 = q3 = lane & 3u; }
        const float4* p = tab + 4u * size_t(rec);
        float4 a, b, c, d;
        if (mode == 5)
        {
            // 1 KB block per wave-instruction: lane i reads 16 B at 16 i (4 instructions, 4 KB)
            const float4* blk = tab + 4u * size_t(__shfl(link, 0) & ~63u);
            a = blk[lane]; b = blk[64u + lane]; c = blk[128u + lane]; d = blk[192u + lane];
        }
        else { a = p[q0]; b = p[q1]; c = p[q2]; d = p[q3]; }
        acc += a.x + b.y + c.z + d.w;
        // the next record depends on the data (like a child link): hash of the loaded bits
        link = (__float_as_uint(a.x) ^ __float_as_uint(d.w) ^ (link * 0x9E3779B1u)) % nrec;
    }
    if (acc == 1234.5f) out[0] = acc;
}

int main(int argc, char** argv)
{
    const size_t mb = argc > 1 ? size_t(atoi(argv[1])) : 16;
    const int wpc = argc > 2 ? atoi(argv[2]) : 20;
    const int iters = argc > 3 ? atoi(argv[3]) : 2048;
    const uint32_t nrec = uint32_t(mb * 1024 * 1024 / 64);
    std::vector<float> h(size_t(nrec) * 16);
    std::mt19937 g(7);
    for (auto& x : h) x = float(g() & 0xFFFFF) * 1e-3f;
    float4* d = nullptr;
    float* o = nullptr;
    if (hipMalloc(&d, h.size() * 4) != hipSuccess || hipMalloc(&o, 4) != hipSuccess) { fprintf(stderr, "alloc\n"); return 1; }
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    int cus = 0, clk_khz = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const int blocks = cus * wpc / 4;            // 256-thread blocks = 4 waves
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char* names[] = { "per-lane", "pair", "quad", "quad-bcast", "wave", "coalesced" };
    const double lines[] = { 64, 32, 16, 16, 1, 8 };
    for (int mode = 0; mode < 6; ++mode)
    {
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, d, nrec, mode, iters / 8, o);   // warm
        hipEventRecord(a);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(256), 0, 0, d, nrec, mode, iters, o);
        hipEventRecord(b);
        if (hipEventSynchronize(b) != hipSuccess) { fprintf(stderr, "kernel failed\n"); return 1; }
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        const double instr = double(blocks) * 4 * iters * 4;      // wave-level load instructions
        const double cyc = ms * 1e-3 * clk_khz * 1e3;             // at the reported clock
        printf("{\"mode\":\"%s\",\"table_mb\":%zu,\"waves_per_cu\":%d,\"ms\":%.4f,\"wave_loads_per_s\":%.4e,"
               "\"lane_loads_per_s\":%.4e,\"model_lines_per_instr\":%.0f,\"model_lines_per_cu_cycle\":%.4f,"
               "\"clock_mhz\":%d,\"cus\":%d}\n",
               names[mode], mb, wpc, ms, instr / (ms * 1e-3), instr * 64 / (ms * 1e-3), lines[mode],
               instr * lines[mode] / cus / cyc, clk_khz / 1000, cus);
    }
    return 0;
}
