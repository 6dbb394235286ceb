// include/visionaray_hip/detail/vrh_libm.h -- single-precision sin / cos with the results of the host
// C library the reference runs on, for host AND device code.
//
// The reference's cosine_sample_hemisphere (sampling.h:61-71) calls cos / sin on a float, which on
// the CPU is glibc's sinf / cosf.  The device's own cosf / sinf (ocml) round differently in a few
// ulps' worth of cases, which moves an AO direction and, rarely, flips an occlusion test.  These
// functions restate glibc 2.35's single-precision sinf / cosf (sysdeps/ieee754/flt-32/s_sinf.c,
// s_cosf.c, sincosf.h, sincosf_data.c: range reduction in double, polynomials in double, one final
// rounding to float) exactly as the x86_64 library selects them on a CPU with FMA + AVX2 (the
// __sinf_fma / __cosf_fma variants, compiled with a*b+c contracted to fma): every multiply-add the
// FMA build fuses is an explicit fma() here, every other operation is a separate IEEE double
// operation.  No plain product here feeds an addition, so floating-point contraction (any
// -ffp-contract setting of the including translation unit) has nothing to fuse.  Double fma, multiply, add and the conversions are
// correctly rounded on gfx950 as on x86_64, so host and device give the same float.
//
// Checked exhaustively -- every one of the 2^32 float inputs, sinf and cosf -- against the build
// container's libm (tests/test_libm_sincosf.py, tools/libm_check.cpp); the device build against the
// host restatement on the GPU (tests/test_gpu_libm.py).  The one difference left is the NaN returned
// for an infinite input (x86 produces the negative default NaN, the GPU the positive one).
#pragma once

#include <cstdint>
#include <cstring>

#if defined(__HIP__)
#define VRH_LIBM_FN __host__ __device__ inline
#else
#define VRH_LIBM_FN inline
#endif

namespace vrh {
namespace libm {

struct sincos_table
{
    double sign[4];
    double hpi_inv;   // 2 / pi * 2^24 (the quadrant ends up in bits 24..31)
    double hpi;       // pi / 2
    double c0, c1, s1, c2, s2, c3, s3, c4;   // glibc's field order (cosine / sine polynomials)
};

// __sincosf_table[2] (sincosf_data.c): [1] has the cosine polynomial negated (quadrants 2 and 3)
VRH_LIBM_FN const sincos_table& table(int k)
{
    static constexpr sincos_table t[2] = {
        { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
          0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
          0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16 },
        { { 1.0, -1.0, -1.0, 1.0 }, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
          -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
          0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16 },
    };
    return t[k];
}

VRH_LIBM_FN uint32_t asuint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
VRH_LIBM_FN uint32_t abstop12(float f) { return (asuint(f) >> 20) & 0x7ff; }
VRH_LIBM_FN double fmad(double a, double b, double c) { return __builtin_fma(a, b, c); }

// sinf_poly (sincosf.h): n even -> sine polynomial, odd -> cosine polynomial
VRH_LIBM_FN float poly(double x, double x2, const sincos_table& p, int n)
{
    if ((n & 1) == 0)
    {
        const double x3 = x * x2;
        const double s1 = fmad(x2, p.s3, p.s2);
        const double x7 = x3 * x2;
        const double s = fmad(x3, p.s1, x);
        return (float)fmad(x7, s1, s);
    }
    const double x4 = x2 * x2;
    const double c2 = fmad(x2, p.c4, p.c3);
    const double c1 = fmad(x2, p.c1, p.c0);
    const double x6 = x4 * x2;
    const double c = fmad(x4, p.c2, c1);
    return (float)fmad(x6, c2, c);
}

// reduce_fast (|x| < 120): x - n pi/2 with n from the prescaled product, one fused multiply-subtract
VRH_LIBM_FN double reduce_fast(double x, const sincos_table& p, int& n)
{
    const double r = x * p.hpi_inv;
    n = ((int32_t)r + 0x800000) >> 24;
    return fmad(-(double)n, p.hpi, x);
}

// reduce_large: Payne-Hanek with the 2/pi bits of __inv_pio4 (sincosf_data.c)
VRH_LIBM_FN double reduce_large(uint32_t xi, int& np)
{
    static constexpr uint32_t inv_pio4[24] = {
        0xa2, 0xa2f9, 0xa2f983, 0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
        0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
        0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041 };
    const uint32_t* arr = &inv_pio4[(xi >> 26) & 15];
    const int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = (uint64_t)(uint32_t)(xi * arr[0]);
    const uint64_t res1 = (uint64_t)xi * arr[4];
    const uint64_t res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    const uint64_t n = (res0 + (1ull << 61)) >> 62;
    res0 -= n << 62;
    const double x = (double)(int64_t)res0;
    np = (int)n;
    return x * 0x1.921fb54442d18p-62;
}

VRH_LIBM_FN float invalid(float y) { return (y - y) / (y - y); }

// glibc s_sinf.c
VRH_LIBM_FN float sinf(float y)
{
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f))       // |y| < pi / 4
    {
        const double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return poly(x, s, table(0), 0);
    }
    if (abstop12(y) < abstop12(120.0f))
    {
        x = reduce_fast(x, table(0), n);
        const double s = table(0).sign[n & 3];
        return poly(x * s, x * x, table((n & 2) ? 1 : 0), n);
    }
    if (abstop12(y) < abstop12(__builtin_inff()))
    {
        const uint32_t xi = asuint(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, n);
        const double s = table(0).sign[(n + sign) & 3];
        return poly(x * s, x * x, table(((n + sign) & 2) ? 1 : 0), n);
    }
    return invalid(y);
}

// glibc s_cosf.c
VRH_LIBM_FN float cosf(float y)
{
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921fb6p-1f))
    {
        const double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return poly(x, x2, table(0), 1);
    }
    if (abstop12(y) < abstop12(120.0f))
    {
        x = reduce_fast(x, table(0), n);
        const double s = table(0).sign[n & 3];
        return poly(x * s, x * x, table((n & 2) ? 1 : 0), n ^ 1);
    }
    if (abstop12(y) < abstop12(__builtin_inff()))
    {
        const uint32_t xi = asuint(y);
        const int sign = (int)(xi >> 31);
        x = reduce_large(xi, n);
        const double s = table(0).sign[(n + sign) & 3];
        return poly(x * s, x * x, table(((n + sign) & 2) ? 1 : 0), n ^ 1);
    }
    return invalid(y);
}

} // namespace libm
} // namespace vrh

#undef VRH_LIBM_FN
