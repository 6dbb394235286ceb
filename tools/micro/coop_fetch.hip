// Microbenchmark: per-lane 64-B record fetch (4 x dwordx4 per lane, 64 records per wave-load) vs a
// cooperative fetch (lane row r loads quarter r of the records of its 4-lane column group, then a
// 4x4 transpose with v_permlane32_swap / v_permlane16_swap), a quad-cooperative fetch transposed with
// DPP, and the same quad fetch transposed through LDS (register-staged: ds_write + ds_read; or
// global_load_lds_dwordx4 straight into LDS + ds_read): dependent chains of random records.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <random>

__device__ __forceinline__ void tr4(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3)
{
    auto s02 = __builtin_amdgcn_permlane32_swap(a0, a2, false, false); a0 = s02[0]; a2 = s02[1];
    auto s13 = __builtin_amdgcn_permlane32_swap(a1, a3, false, false); a1 = s13[0]; a3 = s13[1];
    auto s01 = __builtin_amdgcn_permlane16_swap(a0, a1, false, false); a0 = s01[0]; a1 = s01[1];
    auto s23 = __builtin_amdgcn_permlane16_swap(a2, a3, false, false); a2 = s23[0]; a3 = s23[1];
}
__device__ __forceinline__ void tr4f(float4& a0, float4& a1, float4& a2, float4& a3)
{
#define TRC(c) { uint32_t x0 = __float_as_uint(a0.c), x1 = __float_as_uint(a1.c), x2 = __float_as_uint(a2.c), x3 = __float_as_uint(a3.c); \
                 tr4(x0, x1, x2, x3); a0.c = __uint_as_float(x0); a1.c = __uint_as_float(x1); a2.c = __uint_as_float(x2); a3.c = __uint_as_float(x3); }
    TRC(x) TRC(y) TRC(z) TRC(w)
#undef TRC
}

// 4x4 transpose inside each quad of lanes (lane 4k + m): a_j on lane m -> a_m on lane j, two
// exchange stages with DPP quad_perm (partner at distance 2, then 1) and selects
template <int CTRL>
__device__ __forceinline__ uint32_t qx(uint32_t v) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ void qtr4(uint32_t& a0, uint32_t& a1, uint32_t& a2, uint32_t& a3, uint32_t lane)
{
    const bool b1 = (lane & 2u) != 0u, b0 = (lane & 1u) != 0u;
    // stage 1 (distance 2): pairs (a0, a2), (a1, a3)
    uint32_t s = b1 ? a0 : a2, r = qx<0x4E>(s);
    if (b1) a0 = r; else a2 = r;
    s = b1 ? a1 : a3; r = qx<0x4E>(s);
    if (b1) a1 = r; else a3 = r;
    // stage 2 (distance 1): pairs (a0, a1), (a2, a3)
    s = b0 ? a0 : a1; r = qx<0xB1>(s);
    if (b0) a0 = r; else a1 = r;
    s = b0 ? a2 : a3; r = qx<0xB1>(s);
    if (b0) a2 = r; else a3 = r;
}
__device__ __forceinline__ void qtr4f(float4& a0, float4& a1, float4& a2, float4& a3, uint32_t lane)
{
#define TRC(c) { uint32_t x0 = __float_as_uint(a0.c), x1 = __float_as_uint(a1.c), x2 = __float_as_uint(a2.c), x3 = __float_as_uint(a3.c); \
                 qtr4(x0, x1, x2, x3, lane); a0.c = __uint_as_float(x0); a1.c = __uint_as_float(x1); a2.c = __uint_as_float(x2); a3.c = __uint_as_float(x3); }
    TRC(x) TRC(y) TRC(z) TRC(w)
#undef TRC
}

__global__ __launch_bounds__(64) void chase(const float4* __restrict__ tab, uint32_t mask, int coop, int iters,
                                            uint32_t* out)
{
    // LDS staging of the quad fetch: load j lands in region j (lane-linear, 16 B per lane);
    // lane 4k + j then reads its record as 64 contiguous bytes of region j at slot 4k
    __shared__ float4 stage[4][64];
    const uint32_t lane = threadIdx.x & 63u, row = lane >> 4;
    uint32_t link = (blockIdx.x * 64u + lane) * 2654435761u & mask;
    float acc = 0.0f;
    for (int i = 0; i < iters; ++i)
    {
        float4 q0, q1, q2, q3;
        if (!coop)
        {
            const float4* p = tab + 4u * link;
            q0 = p[0]; q1 = p[1]; q2 = p[2]; q3 = p[3];
        }
        else if (coop == 2)
        {
            uint32_t l0 = link, l1 = link, l2 = link, l3 = link;
            qtr4(l0, l1, l2, l3, lane);                // l_j = link of quad lane j
            const uint32_t m = lane & 3u;
            q0 = tab[4u * l0 + m]; q1 = tab[4u * l1 + m]; q2 = tab[4u * l2 + m]; q3 = tab[4u * l3 + m];
            qtr4f(q0, q1, q2, q3, lane);               // q_k = quarter k of my own record
        }
        else if (coop == 3 || coop == 4)
        {
            uint32_t l0 = link, l1 = link, l2 = link, l3 = link;
            qtr4(l0, l1, l2, l3, lane);                // l_j = link of quad lane j
            const uint32_t m = lane & 3u;
            if (coop == 3)
            {
                const float4 a0 = tab[4u * l0 + m], a1 = tab[4u * l1 + m], a2 = tab[4u * l2 + m], a3 = tab[4u * l3 + m];
                stage[0][lane] = a0; stage[1][lane] = a1; stage[2][lane] = a2; stage[3][lane] = a3;
            }
            else
            {
                typedef __attribute__((address_space(1))) void gvoid;
                typedef __attribute__((address_space(3))) void lvoid;
                __builtin_amdgcn_global_load_lds((gvoid*)(tab + 4u * l0 + m), (lvoid*)&stage[0][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gvoid*)(tab + 4u * l1 + m), (lvoid*)&stage[1][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gvoid*)(tab + 4u * l2 + m), (lvoid*)&stage[2][0], 16, 0, 0);
                __builtin_amdgcn_global_load_lds((gvoid*)(tab + 4u * l3 + m), (lvoid*)&stage[3][0], 16, 0, 0);
                __builtin_amdgcn_s_waitcnt(0x0070);    // vmcnt(0) (lgkmcnt/expcnt left at max)
            }
            __builtin_amdgcn_wave_barrier();
            const float4* mine = &stage[m][lane & ~3u];
            q0 = mine[0]; q1 = mine[1]; q2 = mine[2]; q3 = mine[3];
            __builtin_amdgcn_wave_barrier();
        }
        else
        {
            uint32_t l0 = link, l1 = link, l2 = link, l3 = link;
            tr4(l0, l1, l2, l3);                       // l_j = link of row j of my column
            q0 = tab[4u * l0 + row]; q1 = tab[4u * l1 + row]; q2 = tab[4u * l2 + row]; q3 = tab[4u * l3 + row];
            tr4f(q0, q1, q2, q3);                      // q_k = quarter k of my own record
        }
        acc += q0.x + q1.y + q2.z + q3.w;
        link = (__float_as_uint(q0.x) ^ __float_as_uint(q1.y) ^ __float_as_uint(q2.z) ^ __float_as_uint(q3.w)) & mask;
    }
    out[blockIdx.x * 64u + lane] = link ^ __float_as_uint(acc);
}

int main(int argc, char** argv)
{
    const uint32_t nrec = argc > 1 ? (1u << atoi(argv[1])) : (1u << 12);
    std::vector<uint32_t> h(nrec * 16);
    std::mt19937 g(7);
    for (auto& x : h) x = g();
    float4* d; uint32_t *o, *o2;
    (void)hipMalloc(&d, h.size() * 4);
    int cus = 0; (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int iters = 2048, blocks = cus * (argc > 2 ? atoi(argv[2]) : 24);
    (void)hipMalloc(&o, blocks * 64 * 4); (void)hipMalloc(&o2, blocks * 64 * 4);
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    std::vector<uint32_t> r0(blocks * 64), r1(blocks * 64);
    const char* names[] = { "per-lane 4 x dwordx4", "row-cooperative + permlane transpose", "quad-cooperative + DPP transpose",
                            "quad-cooperative + LDS transpose (reg-staged)", "quad-cooperative + global_load_lds + LDS read" };
    for (int coop = 0; coop < 5; ++coop)
    {
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, nrec - 1, coop, iters, coop ? o2 : o);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, nrec - 1, coop, iters, coop ? o2 : o);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
        float ms = 0; (void)hipEventElapsedTime(&ms, a, b);
        printf("table %u KB %s: %.3f ms, %.1f record fetches/ns\n", nrec / 16, names[coop],
               ms, double(blocks) * 64 * iters / (ms * 1e6));
        if (coop) { (void)hipMemcpy(r1.data(), o2, r1.size() * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(r0.data(), o, r0.size() * 4, hipMemcpyDeviceToHost); printf("  same results as per-lane: %s\n", r0 == r1 ? "yes" : "NO"); }
    }
    return 0;
}
