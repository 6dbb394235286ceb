// include/visionaray_hip/reference.h -- the reference's own Visionaray headers as host AND device
// code in a translation unit compiled by hipcc.
//
// The reference marks its functions VSNRAY_FUNC / MATH_FUNC, which are `__device__ __host__` only
// for nvcc (detail/macros.h:47-53, math/config.h:24-25); compiled by hipcc they would be host-only.
// This header includes them inside clang's `#pragma clang force_cuda_host_device` region, which
// gives every declaration in it both attributes -- the reference's vector / ray / primitive types,
// intersect(), closest_hit / any_hit / multi_hit (traverse_linear.inl), update_if / is_closer,
// basic_intersector, get_normal / get_tex_coord / get_surface, the materials and lights, simple::
// and whitted::kernel, random_sampler<float> (std::default_random_engine +
// std::uniform_real_distribution<float>, so its draws on the GPU are the CPU's bit for bit) and
// cosine_sample_hemisphere (sampling.h:61-71, whose float sin / cos are the host library's on the device
// too: detail/vrh_libm.h).  No reference source is changed or copied, and no
// CUDA macro is defined: `__CUDACC__` / `__CUDA_ARCH__` stay undefined, so the reference takes the
// same (CPU) code paths it takes under g++.
//
// A Visionaray program written for cuda_sched ports to hip_sched by replacing its Visionaray include
// lines with
//
//     #include <visionaray_hip/reference.h>      // the reference's headers, host + device
//     #include <visionaray_hip/hip_kernels.h>    // hip_sched / hip_index_bvh / hip_buffer_rt
//
// (see INTEGRATION.md §3 for the full list of changed lines).  System and compiler headers must not
// fall inside the region (a host-only libc / intrinsics declaration redeclared as host+device is an
// error), so every one the reference uses is included first; <random> is the exception: it is
// included inside, so that std::linear_congruential_engine and std::uniform_real_distribution
// become device code for random_sampler<float>.
#pragma once

#if !defined(__HIP__)
#error "visionaray_hip/reference.h makes the reference headers device code: compile this translation unit with hipcc"
#endif

#if defined(VSNRAY_BVH_H) || defined(VSNRAY_DETAIL_MACROS_H)
#error "visionaray_hip/reference.h must come before any other Visionaray header"
#endif

#if defined(_GLIBCXX_RANDOM)
#error "visionaray_hip/reference.h must come before <random> (random_sampler<float> needs it as device code)"
#endif

#include <hip/hip_runtime.h>

// the system headers the reference includes, host-only as usual
#include <algorithm>
#include <array>
#include <atomic>
#include <cassert>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <iostream>
#include <istream>
#include <iterator>
#include <limits>
#include <malloc.h>
#include <memory>
#include <mutex>
#include <new>
#include <ostream>
#include <semaphore.h>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "detail/vrh_libm.h"

#pragma clang force_cuda_host_device begin
#include <random>
#include <visionaray/math/math.h>
// sampling.h's sin / cos (cosine_sample_hemisphere, uniform_sample_hemisphere: sampling.h:51-71) on a
// float return what the host C library returns -- on the device through the restatement of glibc's
// sinf / cosf (detail/vrh_libm.h, equal to the host library on every float input), on the host the
// library itself -- so a device AO kernel draws the reference CPU run's directions bit for bit.  Every
// other argument type keeps the reference's own overloads.  sampling.h is included here, first, with
// its two calls renamed; its include guard keeps later includes (brdf.h, kernels.h) from repeating it.
namespace visionaray
{
inline float vrh_libm_cos(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ::vrh::libm::cosf(x);
#else
    return ::cosf(x);
#endif
}
inline float vrh_libm_sin(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return ::vrh::libm::sinf(x);
#else
    return ::sinf(x);
#endif
}
template <typename T> inline auto vrh_libm_cos(T const& x) -> decltype(cos(x)) { return cos(x); }
template <typename T> inline auto vrh_libm_sin(T const& x) -> decltype(sin(x)) { return sin(x); }
} // visionaray
#define cos vrh_libm_cos
#define sin vrh_libm_sin
#include <visionaray/sampling.h>
#undef cos
#undef sin
#include <visionaray/aligned_vector.h>
#include <visionaray/bvh.h>
#include <visionaray/camera.h>
#include <visionaray/get_color.h>
#include <visionaray/get_normal.h>
#include <visionaray/get_shading_normal.h>
#include <visionaray/get_surface.h>
#include <visionaray/get_tex_coord.h>
#include <visionaray/intersector.h>
#include <visionaray/kernels.h>
#include <visionaray/material.h>
#include <visionaray/point_light.h>
#include <visionaray/random_sampler.h>
#include <visionaray/result_record.h>
#include <visionaray/sampling.h>
#include <visionaray/scheduler.h>
#include <visionaray/traverse.h>
#include <visionaray/update_if.h>
#pragma clang force_cuda_host_device end

#define VRH_REFERENCE_HEADERS 1
