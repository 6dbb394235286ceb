// include/visionaray_hip/hip_backend.h -- C++ drop-in of the MI355X traversal backend.
//
// Header-only layer over the C-ABI (include/vrh.h, libvrh.so) that presents Visionaray's scheduler
// / render-target / BVH interface, so application code written for the reference's CUDA path
//
//     cuda_index_bvh<P>  device_bvh(host_bvh);                       // bvh.h:443-448
//     gpu_buffer_rt<PF_RGBA32F, PF_UNSPECIFIED> rt;  rt.resize(w, h); // gpu_buffer_rt.h:19-51
//     cuda_sched<ray> sched;                                          // cuda_sched.h:25-40
//     sched.frame(kernel, make_sched_params(pixel_sampler::uniform_type{}, cam, rt));
//
// ports by renaming the three types to hip_index_bvh / hip_buffer_rt / hip_sched and passing one of
// the built-in kernels (make_hip_closest_hit_kernel / make_hip_ao_kernel) instead of a lambda --
// an arbitrary C++ callable cannot cross a C ABI (hard part 6).
//
// The templates only assume the reference's concepts, so they work with the reference's own types
// (camera, sched_params, index_bvh_t, basic_triangle, basic_sphere) and with the minimal standalone
// types of visionaray_hip/standalone.h:
//   camera       : eye(), center(), up() (vec3 with .x .y .z), fovy(), aspect()       camera.h:46-95
//   sched params : .cam (camera by value), .rt (render target by reference)             scheduler.h:52-75
//   host BVH     : nodes(), indices(), primitives() contiguous containers; 32-B nodes,
//                  64-B basic_triangle<3,float> or 48-B basic_sphere<float> primitives  bvh.h:317-403
//
// Errors: HIP / argument errors surface as visionaray::hip_error (the reference throws
// visionaray::exception from host code, exception.h).
#pragma once

#include "../vrh.h"

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

namespace visionaray
{

// the reference's pixel samplers (sched_common.h:34-50), declared here so that hip_sched can read
// sched_params::pixel_sampler_type (defined by the reference's headers or by standalone.h)
namespace pixel_sampler
{
template <size_t NumSamples> struct ssaa_type;
struct jittered_type;
struct jittered_blend_type;
}

// normal binding tags of make_kernel_params (tags.h:46-47), declared here so the shading kernel
// factory can take them; the reference's (or standalone.h's) definitions complete them
struct normals_per_face_binding;
struct normals_per_vertex_binding;

struct hip_error : std::runtime_error
{
    int status;
    hip_error(const char* what, int s)
        : std::runtime_error(std::string(what) + " failed (status " + std::to_string(s) + "): " + vrh_last_error())
        , status(s)
    {
    }
};

namespace hip_detail
{
inline void check(int rc, const char* what)
{
    if (rc != VRH_OK) throw hip_error(what, rc);
}

// the deepest BVH this process has taken a ref of (hip_index_bvh::ref): a user-kernel launch
// (visionaray_hip/hip_kernels.h) gives its threads the short LDS stack while every such BVH fits it
inline std::atomic<uint32_t>& user_ref_depth()
{
    static std::atomic<uint32_t> d{ 0u };
    return d;
}
inline void note_ref_depth(uint32_t depth)
{
    auto& d = user_ref_depth();
    uint32_t cur = d.load(std::memory_order_relaxed);
    while (depth > cur && !d.compare_exchange_weak(cur, depth, std::memory_order_release, std::memory_order_relaxed)) {}
}

template <typename T, typename = void> struct is_sphere : std::false_type {};
template <typename T> struct is_sphere<T, decltype((void)std::declval<T>().radius)> : std::true_type {};
template <typename T, typename = void> struct is_triangle : std::false_type {};
template <typename T> struct is_triangle<T, decltype((void)std::declval<T>().e2)> : std::true_type {};

// sched_params::scissor_box (scheduler.h:25-31; make_sched_params sets recti(0, 0, w, h), :175),
// read as cuda_sched reads it (cuda_sched.inl:71): x <= px < w, y <= py < h
template <typename SP, typename = void> struct has_scissor : std::false_type {};
template <typename SP> struct has_scissor<SP, decltype((void)std::declval<SP>().scissor_box)> : std::true_type {};

// user kernels (callables) are device code: visionaray_hip/hip_kernels.h, compiled by hipcc,
// specialises this for them; without it hip_sched::frame accepts only the built-in kernels
template <typename K, typename = void>
struct user_kernels
{
    static constexpr bool available = false;
};

// pixel sampler of a sched_params (sched_params::pixel_sampler_type; uniform when it has none) and
// its vrh_pixel_sampler
template <typename T> struct sampler_desc { static constexpr bool supported = false; static constexpr uint32_t kind = 0, count = 0; };
template <size_t N> struct sampler_desc<pixel_sampler::ssaa_type<N>>
{
    static constexpr bool supported = N == 1 || N == 2 || N == 4 || N == 8;
    static constexpr uint32_t kind = N == 1 ? VRH_SAMPLER_UNIFORM : VRH_SAMPLER_SSAA, count = uint32_t(N);
};
template <> struct sampler_desc<pixel_sampler::jittered_type>
{
    static constexpr bool supported = true;
    static constexpr uint32_t kind = VRH_SAMPLER_JITTERED, count = 0;
};
template <> struct sampler_desc<pixel_sampler::jittered_blend_type>
{
    static constexpr bool supported = true;
    static constexpr uint32_t kind = VRH_SAMPLER_JITTERED_BLEND, count = 0;
};
template <typename SP, typename = void> struct sampler_of { using type = pixel_sampler::ssaa_type<1>; };
template <typename SP> struct sampler_of<SP, decltype((void)std::declval<typename SP::pixel_sampler_type*>())>
{
    using type = typename SP::pixel_sampler_type;
};
// sched_params with an intersector (scheduler.h:33-45, 177-193)
template <typename SP, typename = void> struct has_sched_intersector : std::false_type {};
template <typename SP> struct has_sched_intersector<SP, decltype((void)std::declval<typename SP::has_intersector*>())>
    : std::true_type {};

// sched_params with view / projection matrices instead of a camera (scheduler.h:76-96, 197-231)
template <typename SP, typename = void> struct has_camera_matrices : std::false_type {};
template <typename SP> struct has_camera_matrices<SP, decltype((void)std::declval<typename SP::has_camera_matrices*>())>
    : std::true_type {};

template <typename SP> constexpr bool uniform_sampler()
{
    return sampler_desc<typename sampler_of<SP>::type>::kind == VRH_SAMPLER_UNIFORM;
}

template <typename SP>
void set_scissor(SP const& sp, vrh_camera& c)
{
    if constexpr (has_scissor<SP>::value)
    {
        auto const& sb = sp.scissor_box;
        c.scissor[0] = uint32_t(sb.x > 0 ? sb.x : 0);
        c.scissor[1] = uint32_t(sb.y > 0 ? sb.y : 0);
        c.scissor[2] = uint32_t(sb.w > 0 ? sb.w : 0);
        c.scissor[3] = uint32_t(sb.h > 0 ? sb.h : 0);
        // recti(0, 0, 0, 0) is an empty box for the reference, but all-zero means "whole image" in
        // the C ABI: pass the same empty pixel set as (1, 1, 1, 1)
        if (c.scissor[0] == 0 && c.scissor[1] == 0 && c.scissor[2] == 0 && c.scissor[3] == 0)
            c.scissor[0] = c.scissor[1] = c.scissor[2] = c.scissor[3] = 1u;
    }
}
} // hip_detail

//-------------------------------------------------------------------------------------------------
// hip_context: one GPU (HIP device + stream).  Shared by the objects created on it.
//

class hip_context
{
public:
    explicit hip_context(int device = 0, void* hip_stream = nullptr)
    {
        vrh_ctx* c = nullptr;
        hip_detail::check(hip_stream ? vrh_ctx_create_on_stream(device, hip_stream, &c) : vrh_ctx_create(device, &c),
                          "vrh_ctx_create");
        ctx_.reset(c, [](vrh_ctx* p) { vrh_ctx_destroy(p); });
    }
    vrh_ctx* get() const { return ctx_.get(); }
    void sync() const { hip_detail::check(vrh_sync(get()), "vrh_sync"); }
    void set_option(uint32_t opt, int64_t value)
    {
        hip_detail::check(vrh_ctx_set_option(get(), opt, value), "vrh_ctx_set_option");
        if (opt == VRH_OPT_ASYNC_FRAMES) async_frames_ = value != 0;
    }
    // cuda_sched's issue model (cuda_sched.inl:306-320): hip_sched::frame returns once the frame is
    // issued; back-to-back frames overlap their launch tails on the context's frame lanes, and
    // hip_buffer_rt::download / sync() wait for them (vrh.h VRH_OPT_ASYNC_FRAMES)
    void set_async_frames(bool on) { set_option(VRH_OPT_ASYNC_FRAMES, on ? 1 : 0); }
    bool async_frames() const { return async_frames_; }
    vrh_frame_stats last_frame_stats() const
    {
        vrh_frame_stats s{};
        hip_detail::check(vrh_last_frame_stats(get(), &s), "vrh_last_frame_stats");
        return s;
    }

    // device memory that hipcc-compiled launches keep with the context (hip_kernels.h: the logs of
    // VRH_USER_DEFER), allocated and grown there; freed with the context
    struct scratch_block
    {
        std::shared_ptr<void> mem;
        size_t bytes = 0;
    };
    scratch_block& scratch() { return *scratch_; }

    static std::shared_ptr<hip_context> const& default_context()
    {
        static std::shared_ptr<hip_context> d = std::make_shared<hip_context>(0);
        return d;
    }

private:
    std::shared_ptr<vrh_ctx> ctx_;
    bool async_frames_ = false;
    std::shared_ptr<scratch_block> scratch_ = std::make_shared<scratch_block>();
};

//-------------------------------------------------------------------------------------------------
// hip_render_group: several GPUs rendering one frame together (vrh.h vrh_group_*): image-tile
// shards on every device, gathered to device 0 over RCCL.  One process driving every GPU:
// hip_render_group(devices) (ncclCommInitAll); one process per GPU: hip_render_group(ctx, nranks,
// rank, id) with the id from hip_render_group::unique_id() on rank 0.
//

class hip_render_group
{
public:
    // every visible device (devices empty) or the given ones; member i renders on devices[i]
    explicit hip_render_group(std::vector<int> devices = {})
    {
        if (devices.empty())
        {
            int n = 0;
            hip_detail::check(vrh_device_count(&n), "vrh_device_count");
            for (int d = 0; d < n; ++d) devices.push_back(d);
        }
        std::vector<vrh_ctx*> raw;
        for (int d : devices)
        {
            ctxs_.push_back(std::make_shared<hip_context>(d));
            raw.push_back(ctxs_.back()->get());
        }
        std::vector<vrh_group*> g(raw.size(), nullptr);
        hip_detail::check(vrh_group_create_local(uint32_t(raw.size()), raw.data(), g.data()), "vrh_group_create_local");
        for (auto* p : g) groups_.emplace_back(p, [](vrh_group* q) { vrh_group_free(q); });
    }

    // one rank of a group spread over processes
    // (timeout_ms: the deadline of every wait on a peer, 0 = VRH_GROUP_TIMEOUT_MS; a missed one throws
    // hip_error with VRH_ERR_TIMEOUT after aborting the communicator, vrh_group_join_timeout)
    hip_render_group(std::shared_ptr<hip_context> ctx, uint32_t nranks, uint32_t rank, vrh_group_id const& id,
                     uint32_t timeout_ms = 0)
    {
        vrh_group* g = nullptr;
        hip_detail::check(vrh_group_join_timeout(ctx->get(), nranks, rank, &id, timeout_ms, &g), "vrh_group_join");
        ctxs_.push_back(std::move(ctx));
        groups_.emplace_back(g, [](vrh_group* q) { vrh_group_free(q); });
    }

    static vrh_group_id unique_id()
    {
        vrh_group_id id{};
        hip_detail::check(vrh_group_get_id(&id), "vrh_group_get_id");
        return id;
    }

    size_t size() const { return groups_.size(); }              // members driven by this process
    std::shared_ptr<hip_context> const& context(size_t i) const { return ctxs_[i]; }
    vrh_group* handle(size_t i) const { return groups_[i].get(); }
    bool has_root() const
    {
        for (auto const& g : groups_) { uint32_t r = 1; vrh_group_info(g.get(), nullptr, &r); if (r == 0) return true; }
        return false;
    }
    void sync() const { for (auto const& g : groups_) hip_detail::check(vrh_group_sync(g.get()), "vrh_group_sync"); }

private:
    std::vector<std::shared_ptr<hip_context>> ctxs_;
    std::vector<std::shared_ptr<vrh_group>> groups_;
};

//-------------------------------------------------------------------------------------------------
// hip_bvh_ref: what hip_index_bvh::ref() hands to kernels -- the scene's device arrays
// (vrh_scene_view); closest_hit / any_hit of visionaray_hip/hip_kernels.h traverse it
//

struct hip_bvh_ref
{
    vrh_scene_view view;
};

// the typed ref hip_index_bvh<P>::ref() returns (index_bvh_ref_t<P>, bvh.h:190-235): the same view,
// plus the primitive type, which the reference's traversal templates read as BVH::primitive_type
// when visionaray_hip/reference.h brings them to the device
template <typename Primitive>
struct hip_bvh_ref_t : hip_bvh_ref
{
    using primitive_type = Primitive;
#if defined(__HIP__)
    __host__ __device__ size_t num_primitives() const { return view.num_prims; }   // index_bvh_ref_t::num_primitives
    // primitive i in leaf order (index_bvh_ref_t::primitive, bvh.h:226-229: the device copy holds the
    // primitives already permuted by the index list), device code; defined in visionaray_hip/hip_kernels.h
    __host__ __device__ Primitive primitive(size_t i) const;
#else
    size_t num_primitives() const { return view.num_prims; }
#endif
};

//-------------------------------------------------------------------------------------------------
// hip_index_bvh<P>: device-resident copy of a host index BVH (the cuda_index_bvh copy-ctor)
//

template <typename Primitive>
class hip_index_bvh
{
public:
    using primitive_type = Primitive;
    using bvh_ref = hip_bvh_ref_t<Primitive>;      // cuda_index_bvh<P>::bvh_ref (bvh.h:344)
    static_assert(hip_detail::is_triangle<Primitive>::value || hip_detail::is_sphere<Primitive>::value,
                  "hip_index_bvh supports basic_triangle<3,float> and basic_sphere<float>");

    // host_bvh: index_bvh<P> (nodes(), indices(), primitives()); face_normals: 16-B vec3 per
    // primitive (normals_per_face_binding, get_normal.h:26-37), needed by the AO kernel
    template <typename HostBVH>
    explicit hip_index_bvh(HostBVH const& host_bvh, void const* face_normals = nullptr,
                           std::shared_ptr<hip_context> ctx = hip_context::default_context())
        : ctx_(std::move(ctx))
    {
        static_assert(sizeof(*host_bvh.nodes().data()) == 32, "bvh_node must be 32 bytes");
        static_assert(sizeof(Primitive) == (hip_detail::is_sphere<Primitive>::value ? 48 : 64),
                      "primitive layout must match basic_triangle<3,float> / basic_sphere<float>");
        vrh_scene* s = nullptr;
        hip_detail::check(vrh_scene_upload(ctx_->get(), host_bvh.nodes().data(), uint32_t(host_bvh.nodes().size()),
                                           host_bvh.primitives().data(), uint32_t(host_bvh.primitives().size()),
                                           hip_detail::is_sphere<Primitive>::value ? VRH_PRIM_SPHERE48 : VRH_PRIM_TRI64,
                                           host_bvh.indices().data(), uint32_t(host_bvh.indices().size()),
                                           face_normals, &s),
                          "vrh_scene_upload");
        scene_.reset(s, [](vrh_scene* p) { vrh_scene_free(p); });
    }

    // build<index_bvh<P>> + the copy to the device in one step, on the GPU (vrh_scene_build: linear
    // BVH, leaves of <= max_leaf primitives).  prims: contiguous container of P; face_normals: any
    // container of vec3-likes, one per primitive (may be empty for spheres / primary-only use).
    template <typename Prims, typename Normals>
    static hip_index_bvh gpu_build(Prims const& prims, Normals const& face_normals, uint32_t max_leaf = 4,
                                   std::shared_ptr<hip_context> ctx = hip_context::default_context())
    {
        static_assert(sizeof(*prims.data()) == sizeof(Primitive), "primitive container of the BVH's type");
        std::vector<float> rows;
        rows.reserve(4 * face_normals.size());
        for (auto const& n : face_normals) { rows.push_back(n.x); rows.push_back(n.y); rows.push_back(n.z); rows.push_back(0.0f); }
        if (!rows.empty() && face_normals.size() != prims.size())
            throw hip_error("gpu_build: one face normal per primitive", VRH_ERR_INVALID);
        vrh_build_desc desc{ VRH_BUILD_LBVH, max_leaf };
        vrh_scene* s = nullptr;
        hip_detail::check(vrh_scene_build(ctx->get(), prims.data(), uint32_t(prims.size()),
                                          hip_detail::is_sphere<Primitive>::value ? VRH_PRIM_SPHERE48 : VRH_PRIM_TRI64,
                                          rows.empty() ? nullptr : rows.data(), &desc, &s),
                          "vrh_scene_build");
        return hip_index_bvh(s, std::move(ctx));
    }

    // normals_per_vertex_binding array (get_shading_normal.h:64-84): 3 per primitive, entry
    // 3 * prim_id + k for vertex k; any container of vec3-likes (x, y, z)
    template <typename Normals>
    void set_vertex_normals(Normals const& normals)
    {
        std::vector<float> rows;
        rows.reserve(4 * normals.size());
        for (auto const& n : normals) { rows.push_back(n.x); rows.push_back(n.y); rows.push_back(n.z); rows.push_back(0.0f); }
        hip_detail::check(vrh_scene_set_vertex_normals(handle(), rows.data(), uint32_t(normals.size())),
                          "vrh_scene_set_vertex_normals");
    }

    vrh_scene* handle() const { return scene_.get(); }
    hip_context& context() const { return *ctx_; }

    // the device BVH a kernel traverses (cuda_index_bvh::ref(), bvh.h:344-350): a plain view of
    // the device arrays, passed by value into user kernels (visionaray_hip/hip_kernels.h)
    hip_bvh_ref_t<Primitive> ref() const
    {
        hip_bvh_ref_t<Primitive> r{};
        hip_detail::check(vrh_scene_get_view(handle(), 0, &r.view), "vrh_scene_get_view");
        hip_detail::note_ref_depth(r.view.max_depth);
        return r;
    }

    vrh_scene_info info() const
    {
        vrh_scene_info i{};
        hip_detail::check(vrh_scene_get_info(handle(), &i), "vrh_scene_get_info");
        return i;
    }

    // scene replication over a render group (vrh_group_broadcast_scene): the process
    // holding rank 0 passes its BVH (on rank 0's context), the others nullptr; one replica per
    // member this process drives, on that member's context, broadcast over RCCL instead of built
    // or uploaded once per GPU
    static std::vector<hip_index_bvh> broadcast(hip_render_group const& group, hip_index_bvh const* root_bvh)
    {
        std::vector<vrh_group*> g;
        for (size_t i = 0; i < group.size(); ++i) g.push_back(group.handle(i));
        std::vector<vrh_scene*> out(g.size(), nullptr);
        hip_detail::check(vrh_group_broadcast_scene(uint32_t(g.size()), g.data(), root_bvh ? root_bvh->handle() : nullptr,
                                                    out.data()),
                          "vrh_group_broadcast_scene");
        std::vector<hip_index_bvh> r;
        for (size_t i = 0; i < g.size(); ++i) r.push_back(hip_index_bvh(out[i], group.context(i)));
        return r;
    }

private:
    hip_index_bvh(vrh_scene* s, std::shared_ptr<hip_context> ctx) : ctx_(std::move(ctx))
    {
        scene_.reset(s, [](vrh_scene* p) { vrh_scene_free(p); });
    }

    std::shared_ptr<hip_context> ctx_;
    std::shared_ptr<vrh_scene> scene_;
};

//-------------------------------------------------------------------------------------------------
// hip_index_bvh_list<P>: a list of device BVHs rendered as one scene -- the [begin, end) range of
// bvh_refs that closest_hit / any_hit take (traverse_linear.inl:76-141; ao/main.cpp:171-178 builds
// such a vector).  Every BVH is traversed on its own per ray and merged by is_closer / update_if
// (vrh.h vrh_scene_list_create).  face_normals: one 16-B vec3 per prim_id over the whole list.
//

template <typename Primitive>
class hip_index_bvh_list
{
public:
    using primitive_type = Primitive;

    hip_index_bvh_list(std::vector<hip_index_bvh<Primitive>> const& bvhs, void const* face_normals = nullptr,
                       uint32_t num_normals = 0, std::shared_ptr<hip_context> ctx = hip_context::default_context())
        : ctx_(std::move(ctx))
    {
        std::vector<vrh_scene const*> h;
        for (auto const& b : bvhs) h.push_back(b.handle());
        vrh_scene* s = nullptr;
        hip_detail::check(vrh_scene_list_create(ctx_->get(), h.data(), uint32_t(h.size()), face_normals, num_normals, &s),
                          "vrh_scene_list_create");
        scene_.reset(s, [](vrh_scene* p) { vrh_scene_free(p); });
    }

    vrh_scene* handle() const { return scene_.get(); }
    hip_context& context() const { return *ctx_; }

private:
    std::shared_ptr<hip_context> ctx_;
    std::shared_ptr<vrh_scene> scene_;
};

//-------------------------------------------------------------------------------------------------
// hip_buffer_rt<CF, DF>: gpu_buffer_rt replacement.  Colour is RGBA32F; the render target also
// keeps the closest-hit prim_id / t and the AO occlusion mask (the integer outputs used for parity).
//

template <auto ColorFormat, auto DepthFormat>
class hip_buffer_rt
{
    // the formats of the measured configurations; other formats are a
    // compile error rather than a silent RGBA32F target (values as in pixel_format.h:15-60)
    static_assert(int(ColorFormat) == 12, "hip_buffer_rt: colour format PF_RGBA32F");
    static_assert(int(DepthFormat) == 0, "hip_buffer_rt: depth format PF_UNSPECIFIED (no depth buffer)");

public:
    struct ref_type          // render_target_ref analogue: raw device pointers + size
    {
        float* color;        // RGBA32F
        uint32_t* prim_id;
        float* t;
        uint8_t* occ;
        size_t width, height;
    };

    explicit hip_buffer_rt(std::shared_ptr<hip_context> ctx = hip_context::default_context())
        : ctx_(std::move(ctx))
    {
    }

    void resize(size_t w, size_t h)
    {
        vrh_rt* r = nullptr;
        hip_detail::check(vrh_rt_alloc(ctx_->get(), uint32_t(w), uint32_t(h), VRH_RT_ALL, &r), "vrh_rt_alloc");
        rt_.reset(r, [](vrh_rt* p) { vrh_rt_free(p); });
        width_ = w;
        height_ = h;
    }

    size_t width() const { return width_; }
    size_t height() const { return height_; }

    template <typename Vec4>
    void clear_color_buffer(Vec4 const& c)
    {
        float f[4] = { float(c.x), float(c.y), float(c.z), float(c.w) };
        hip_detail::check(vrh_rt_clear(ctx_->get(), rt_.get(), f), "vrh_rt_clear");
    }
    void clear_color_buffer()
    {
        float f[4] = { 0, 0, 0, 0 };
        hip_detail::check(vrh_rt_clear(ctx_->get(), rt_.get(), f), "vrh_rt_clear");
    }

    void begin_frame() {}
    // end_frame() synchronises, so hip_sched::frame blocks like tiled_sched::frame -- unless the
    // context issues frames asynchronously (hip_context::set_async_frames): then it returns at once,
    // as gpu_buffer_rt::end_frame does (gpu_buffer_rt.inl:84-86), and download() waits
    void end_frame()
    {
        if (!ctx_->async_frames()) ctx_->sync();
    }

    ref_type ref()
    {
        ref_type r{};
        void* c = nullptr;
        hip_detail::check(vrh_rt_get_buffers(rt_.get(), &c, &r.prim_id, &r.t, &r.occ), "vrh_rt_get_buffers");
        r.color = static_cast<float*>(c);
        r.width = width_;
        r.height = height_;
        return r;
    }

    // device -> host copies (display_color_buffer analogue; any pointer may be null)
    void download(float* rgba, uint32_t* prim_id = nullptr, float* t = nullptr, uint8_t* occ = nullptr)
    {
        hip_detail::check(vrh_rt_download(ctx_->get(), rt_.get(), rgba, prim_id, t, occ), "vrh_rt_download");
    }

    // hit lists of multi_hit<N> kernels: entry [pixel * N + k], misses 0xFFFFFFFF / -1
    void enable_multi_hit(unsigned max_hits)
    {
        hip_detail::check(vrh_rt_alloc_multi_hit(ctx_->get(), rt_.get(), max_hits), "vrh_rt_alloc_multi_hit");
    }
    void download_multi_hit(uint32_t* prim_ids, float* t)
    {
        hip_detail::check(vrh_rt_download_multi_hit(ctx_->get(), rt_.get(), prim_ids, t), "vrh_rt_download_multi_hit");
    }

    vrh_rt* handle() const { return rt_.get(); }

private:
    std::shared_ptr<hip_context> ctx_;
    std::shared_ptr<vrh_rt> rt_;
    size_t width_ = 0, height_ = 0;
};

//-------------------------------------------------------------------------------------------------
// Built-in kernels (what a C ABI can carry)
//

struct hip_builtin_kernel
{
    vrh_scene* scene;
    vrh_kernel_desc desc;
};

template <typename BVH, typename Vec4>
hip_builtin_kernel make_hip_closest_hit_kernel(BVH const& bvh, Vec4 const& bg)
{
    // closest_hit(ray, bvhs) (traverse_linear.inl:286-329); colour = hit ? 1 : bg
    hip_builtin_kernel k{ bvh.handle(), {} };
    k.desc.kind = VRH_KERNEL_PRIMARY;
    k.desc.bg[0] = bg.x; k.desc.bg[1] = bg.y; k.desc.bg[2] = bg.z; k.desc.bg[3] = bg.w;
    return k;
}

template <typename BVH, typename Vec4>
hip_builtin_kernel make_hip_ao_kernel(BVH const& bvh, Vec4 const& bg, unsigned samples = 8, float radius = 0.1f,
                                      float eps = 1e-3f)
{
    // ao/main.cpp:183-246 with the deterministic Appendix-A sampler
    hip_builtin_kernel k{ bvh.handle(), {} };
    k.desc.kind = VRH_KERNEL_AO;
    k.desc.samples = samples;
    k.desc.radius = radius;
    k.desc.eps = eps;
    k.desc.bg[0] = bg.x; k.desc.bg[1] = bg.y; k.desc.bg[2] = bg.z; k.desc.bg[3] = bg.w;
    // ao/main.cpp takes AO_Samples from its command line (main.cpp:85, 115): with more than 8 the
    // per-sample mask no longer fits hip_buffer_rt's occlusion byte, which is then left untouched
    // (the colour carries the result, as in the reference, which has no such buffer)
    if (samples > 8u) k.desc.flags |= VRH_KERNEL_NO_OCC;
    return k;
}

//-------------------------------------------------------------------------------------------------
// Shading: materials + lights of make_kernel_params (kernels.h:357-389)
// on the device, and the simple::kernel (detail/simple.inl:19-83) built-in.
//

namespace hip_detail
{
template <typename S, typename = void> struct has_samples : std::false_type {};
template <typename S> struct has_samples<S, decltype((void)std::declval<S>().samples())> : std::true_type {};

// rgb of a spectrum<float> (RGB spectrum: samples() is a vec3, spectrum.h:25-36) or of a vec3
template <typename S>
void rgb(S const& s, float out[3])
{
    if constexpr (has_samples<S>::value) { auto v = s.samples(); out[0] = v.x; out[1] = v.y; out[2] = v.z; }
    else { out[0] = s.x; out[1] = s.y; out[2] = s.z; }
}

// plastic<float> through its getters (material.h:297-316)
template <typename M>
vrh_plastic to_plastic(M const& m)
{
    vrh_plastic p{};
    rgb(m.get_ca(), p.ca); p.ka = m.get_ka();
    rgb(m.get_cd(), p.cd); p.kd = m.get_kd();
    rgb(m.get_cs(), p.cs); p.ks = m.get_ks();
    p.exp = m.get_specular_exp();
    return p;
}
inline vrh_plastic to_plastic(vrh_plastic const& m) { return m; }

// point_light<float> (point_light.h:18-66) has no cl / kl getters; with the default constant
// attenuation 1, intensity(position()) is exactly cl * kl (point_light.inl:12-28).  Other
// attenuations: pass vrh_point_light records instead.
template <typename L>
vrh_point_light to_point_light(L const& l)
{
    if (l.constant_attenuation() != 1.0f)
        throw hip_error("point_light with constant attenuation != 1: pass vrh_point_light records", VRH_ERR_INVALID);
    vrh_point_light r{};
    auto pos = l.position();
    r.position[0] = pos.x; r.position[1] = pos.y; r.position[2] = pos.z;
    auto i = l.intensity(pos);
    r.cl[0] = i.x; r.cl[1] = i.y; r.cl[2] = i.z;
    r.kl = 1.0f;
    r.constant_att = 1.0f;
    r.linear_att = l.linear_attenuation();
    r.quadratic_att = l.quadratic_attenuation();
    return r;
}
inline vrh_point_light to_point_light(vrh_point_light const& l) { return l; }

inline uint32_t binding_of(normals_per_face_binding const&) { return VRH_NORMALS_PER_FACE; }
inline uint32_t binding_of(normals_per_vertex_binding const&) { return VRH_NORMALS_PER_VERTEX; }
} // hip_detail

// device materials (plastic, indexed by geom_id) and point lights
class hip_shading
{
public:
    template <typename Materials, typename Lights>
    hip_shading(Materials const& materials, Lights const& lights,
                std::shared_ptr<hip_context> ctx = hip_context::default_context())
        : ctx_(std::move(ctx))
    {
        std::vector<vrh_plastic> m;
        for (auto const& x : materials) m.push_back(hip_detail::to_plastic(x));
        std::vector<vrh_point_light> l;
        for (auto const& x : lights) l.push_back(hip_detail::to_point_light(x));
        vrh_shading* s = nullptr;
        hip_detail::check(vrh_shading_create(ctx_->get(), m.data(), uint32_t(m.size()), l.data(), uint32_t(l.size()), &s),
                          "vrh_shading_create");
        shading_.reset(s, [](vrh_shading* p) { vrh_shading_free(p); });
    }

    vrh_shading* handle() const { return shading_.get(); }

private:
    std::shared_ptr<hip_context> ctx_;
    std::shared_ptr<vrh_shading> shading_;
};

// Mask intersector (vrh_hit_mask_create): what the intersector example's mask_intersector
// (examples/intersector/main.cpp:251-330, a basic_intersector clearing hr.hit from a mask over the
// hit's texture coordinate) does, with the mask given as data.  tex_coords: 3 per prim_id (the
// model's tex_coords, any type with .x / .y); mask: w x h bytes, row-major.
class hip_hit_mask
{
public:
    template <typename TexCoords>
    hip_hit_mask(TexCoords const& tex_coords, uint8_t const* mask, unsigned w, unsigned h,
                 std::shared_ptr<hip_context> ctx = hip_context::default_context())
        : ctx_(std::move(ctx))
    {
        std::vector<float> tc;
        tc.reserve(2 * tex_coords.size());
        for (auto const& c : tex_coords) { tc.push_back(c.x); tc.push_back(c.y); }
        vrh_hit_mask* m = nullptr;
        hip_detail::check(vrh_hit_mask_create(ctx_->get(), tc.data(), uint32_t(tex_coords.size()), mask, w, h, &m),
                          "vrh_hit_mask_create");
        mask_.reset(m, [](vrh_hit_mask* p) { vrh_hit_mask_free(p); });
    }

    vrh_hit_mask* handle() const { return mask_.get(); }

private:
    std::shared_ptr<hip_context> ctx_;
    std::shared_ptr<vrh_hit_mask> mask_;
};

// closest_hit(ray, begin, end, intersector) / any_hit(..., intersector) for every ray of a built-in
// kernel (traverse_linear.inl:232-329): the kernel with the mask intersector attached
inline hip_builtin_kernel with_intersector(hip_builtin_kernel k, hip_hit_mask const& mask)
{
    k.desc.hit_mask = mask.handle();
    return k;
}

// simple::kernel over make_kernel_params(binding, prims, normals, materials, lights, bounces, eps,
// bg, ambient): the normals live in the hip_index_bvh (face normals at upload, per-vertex normals
// via set_vertex_normals), materials / lights in the hip_shading
template <typename NormalBinding, typename BVH, typename Vec4>
hip_builtin_kernel make_hip_simple_kernel(NormalBinding const& binding, BVH const& bvh, hip_shading const& shading,
                                          Vec4 const& bg, Vec4 const& ambient)
{
    hip_builtin_kernel k{ bvh.handle(), {} };
    k.desc.kind = VRH_KERNEL_SIMPLE;
    k.desc.bg[0] = bg.x; k.desc.bg[1] = bg.y; k.desc.bg[2] = bg.z; k.desc.bg[3] = bg.w;
    k.desc.ambient[0] = ambient.x; k.desc.ambient[1] = ambient.y; k.desc.ambient[2] = ambient.z;
    k.desc.ambient[3] = ambient.w;
    k.desc.normal_binding = hip_detail::binding_of(binding);
    k.desc.shading = shading.handle();
    return k;
}

// multi_hit<N> (traverse_linear.inl:333-380) with the compositing kernel of the reference's
// multi_hit example (examples/multi_hit/main.cpp:166-235); the N-entry hit lists land in the render
// target (hip_buffer_rt::enable_multi_hit(N), download_multi_hit)
// whitted::kernel (detail/whitted.inl:186-277) over make_kernel_params(binding, prims, normals,
// materials, lights, num_bounces, epsilon, bg, ambient): simple::kernel's shading plus a shadow ray
// per light and the plastic reflection (kr 0.1)
template <typename NormalBinding, typename BVH, typename Vec4>
hip_builtin_kernel make_hip_whitted_kernel(NormalBinding const& binding, BVH const& bvh, hip_shading const& shading,
                                           unsigned num_bounces, float epsilon, Vec4 const& bg, Vec4 const& ambient)
{
    hip_builtin_kernel k = make_hip_simple_kernel(binding, bvh, shading, bg, ambient);
    k.desc.kind = VRH_KERNEL_WHITTED;
    k.desc.num_bounces = num_bounces;
    k.desc.eps = epsilon;
    return k;
}

template <unsigned N, typename NormalBinding, typename BVH, typename Vec4>
hip_builtin_kernel make_hip_multi_hit_kernel(NormalBinding const& binding, BVH const& bvh, hip_shading const& shading,
                                             Vec4 const& bg)
{
    static_assert(N >= 1 && N <= VRH_MAX_HITS, "multi_hit<N>: 1 <= N <= 16");
    hip_builtin_kernel k = make_hip_simple_kernel(binding, bvh, shading, bg, bg);
    k.desc.kind = VRH_KERNEL_MULTI_HIT;
    k.desc.ambient[0] = k.desc.ambient[1] = k.desc.ambient[2] = k.desc.ambient[3] = 0.0f;
    k.desc.max_hits = N;
    return k;
}

//-------------------------------------------------------------------------------------------------
// hip_sched<R>: cuda_sched<R> replacement (persistent-thread HIP kernels, tile work stealing)
//

template <typename R>
class hip_sched
{
public:
    // cuda_sched's issue model by default (cuda_sched.inl:306-320: frame() enqueues and returns,
    // gpu_buffer_rt::end_frame is a no-op, gpu_buffer_rt.inl:84-86): the scheduler turns on its
    // context's asynchronous frames (VRH_OPT_ASYNC_FRAMES), so back-to-back frame() calls overlap their
    // launch tails and hip_buffer_rt::download / hip_context::sync wait for them; async_frames = false
    // keeps a frame() that returns only when the frame is done (tiled_sched's behaviour)
    explicit hip_sched(std::shared_ptr<hip_context> ctx = hip_context::default_context(), bool async_frames = true)
        : ctx_(std::move(ctx))
    {
        ctx_->set_async_frames(async_frames);
    }

    // multi-GPU: frames sharded over a render group; `shards` image-tile shards
    // (0 = one per GPU).  frame() then takes one built-in kernel per member of the group (each
    // made from that member's BVH replica) and a render target on member 0's device.
    explicit hip_sched(hip_render_group& group, unsigned shards = 0)
        : ctx_(group.context(0))
        , group_(&group)
        , shards_(shards)
    {
    }

    template <typename SP>
    void frame(std::vector<hip_builtin_kernel> const& kernels, SP sparams, unsigned frame_num = 0)
    {
        static_assert(hip_detail::uniform_sampler<SP>(), "hip_sched(group)::frame: render groups use pixel_sampler::uniform_type");
        static_assert(!hip_detail::has_camera_matrices<SP>::value, "hip_sched(group)::frame: render groups take a camera");
        if (!group_ || kernels.size() != group_->size())
            throw std::runtime_error("hip_sched::frame: one kernel per member of the render group");
        auto const& cam = sparams.cam;
        auto& rt = sparams.rt;
        float eye[3] = { cam.eye().x, cam.eye().y, cam.eye().z };
        float center[3] = { cam.center().x, cam.center().y, cam.center().z };
        float up[3] = { cam.up().x, cam.up().y, cam.up().z };
        vrh_camera c{};
        hip_detail::check(vrh_make_camera(eye, center, up, cam.fovy(), cam.aspect(), uint32_t(rt.width()),
                                          uint32_t(rt.height()), &c), "vrh_make_camera");
        hip_detail::set_scissor(sparams, c);
        std::vector<vrh_group*> g;
        std::vector<vrh_scene const*> sc;
        std::vector<vrh_kernel_desc> kd;
        for (size_t i = 0; i < kernels.size(); ++i)
        {
            g.push_back(group_->handle(i));
            sc.push_back(kernels[i].scene);
            kd.push_back(kernels[i].desc);
        }
        rt.begin_frame();
        hip_detail::check(vrh_render_sharded(uint32_t(g.size()), g.data(), sc.data(), kd.data(),
                                             group_->has_root() ? rt.handle() : nullptr,
                                             (kd[0].flags & VRH_KERNEL_NO_OCC) ? (VRH_RT_ALL & ~uint32_t(VRH_RT_OCC)) : VRH_RT_ALL,
                                             &c, 1, frame_num,
                                             shards_),
                          "vrh_render_sharded");
        group_->sync();
        rt.end_frame();
    }

    // frame(): rt.begin_frame() -> vrh_render -> rt.end_frame() (cuda_sched.inl:306-320; end_frame
    // syncs).  shard: optional image-tile shard (multi-GPU).
    //
    // K may also be a user kernel -- a callable R -> result_record (or (R, sampler&), (R, x, y)),
    // as cuda_sched runs it (cuda_sched.inl:53-99, sched_common.h:78-120) -- when the translation
    // unit includes visionaray_hip/hip_kernels.h and is compiled by hipcc: it then runs on the GPU
    // over the pixels of the scissor box with the reference's primary rays.
    template <typename K, typename SP>
    void frame(K kernel, SP sparams, unsigned frame_num = 0, vrh_shard const* shard = nullptr)
    {
        if constexpr (!std::is_same<K, hip_builtin_kernel>::value)
        {
            static_assert(hip_detail::user_kernels<K>::available,
                          "hip_sched runs the built-in kernels (make_hip_closest_hit_kernel / make_hip_ao_kernel / "
                          "make_hip_simple_kernel / make_hip_multi_hit_kernel) through the C ABI; a user kernel "
                          "(a callable) is device code: include visionaray_hip/hip_kernels.h and compile with hipcc");
            if (shard) throw std::runtime_error("hip_sched::frame: user kernels render the whole image");
            hip_detail::user_kernels<K>::frame(*ctx_, kernel, sparams, frame_num);
            return;
        }
        else
            frame_builtin(kernel, sparams, frame_num, shard);
    }

private:
    template <typename SP>
    void frame_builtin(hip_builtin_kernel const& kernel, SP& sparams, unsigned frame_num, vrh_shard const* shard)
    {
        using PS = hip_detail::sampler_desc<typename hip_detail::sampler_of<SP>::type>;
        static_assert(PS::supported, "hip_sched: the pixel samplers are uniform_type, jittered_type, "
                                     "jittered_blend_type and ssaa_type<2 / 4 / 8>");
        static_assert(!hip_detail::has_sched_intersector<SP>::value,
                      "hip_sched: a built-in kernel takes its intersector as data (with_intersector(kernel, "
                      "hip_hit_mask)); sched_params with an intersector are for user kernels (hip_kernels.h)");
        auto& rt = sparams.rt;
        if constexpr (hip_detail::has_camera_matrices<SP>::value)
        {
            // make_sched_params(sampler, view_matrix, proj_matrix, rt) (scheduler.h:197-212):
            // the matrix primary rays (sched_common.h:152-176), whole image
            if (shard) throw std::runtime_error("hip_sched::frame: camera matrices render the whole image");
            vrh_view_camera vc{};
            std::memcpy(vc.view, sparams.view_matrix.data(), sizeof(vc.view));
            std::memcpy(vc.proj, sparams.proj_matrix.data(), sizeof(vc.proj));
            vc.width = uint32_t(rt.width());
            vc.height = uint32_t(rt.height());
            vrh_camera c{};
            hip_detail::set_scissor(sparams, c);
            std::memcpy(vc.scissor, c.scissor, sizeof(vc.scissor));
            const vrh_pixel_sampler ps{ PS::kind, PS::count };
            rt.begin_frame();
            hip_detail::check(vrh_render_view(ctx_->get(), kernel.scene, rt.handle(), &vc, &kernel.desc, &ps, frame_num),
                              "vrh_render_view");
            rt.end_frame();
            return;
        }
        else
        {
            auto const& cam = sparams.cam;
            float eye[3] = { cam.eye().x, cam.eye().y, cam.eye().z };
            float center[3] = { cam.center().x, cam.center().y, cam.center().z };
            float up[3] = { cam.up().x, cam.up().y, cam.up().z };
            vrh_camera c{};
            hip_detail::check(vrh_make_camera(eye, center, up, cam.fovy(), cam.aspect(), uint32_t(rt.width()),
                                              uint32_t(rt.height()), &c), "vrh_make_camera");
            hip_detail::set_scissor(sparams, c);
            rt.begin_frame();
            if constexpr (PS::kind == VRH_SAMPLER_UNIFORM)
                hip_detail::check(vrh_render(ctx_->get(), kernel.scene, rt.handle(), &c, &kernel.desc, shard, frame_num),
                                  "vrh_render");
            else
            {
                // jittered / jittered_blend / ssaa<N> (sched_common.h:160-300, 440-720)
                if (shard) throw std::runtime_error("hip_sched::frame: pixel samplers other than uniform render the whole image");
                const vrh_pixel_sampler ps{ PS::kind, PS::count };
                hip_detail::check(vrh_render_sampled(ctx_->get(), kernel.scene, rt.handle(), &c, &kernel.desc, &ps, frame_num),
                                  "vrh_render_sampled");
            }
            rt.end_frame();
        }
    }

public:

    // frames in flight (vrh_render_batch): ONE persistent launch renders cams.size() frames of
    // one scene and kernel (up to VRH_MAX_BATCH), camera f into rows [f * H, (f + 1) * H) of rt,
    // whose height is cams.size() * H, with frame number frame_num + f.  Every frame equals its
    // own frame() call; the launch's tail is paid once instead of once per frame.  Synchronous
    // like frame().
    // A user kernel (hip_kernels.h, hipcc) renders its frames in one persistent launch the same way.
    template <typename K, typename Camera, typename RT>
    void frames(K kernel, std::vector<Camera> const& cams, RT& rt, unsigned frame_num = 0)
    {
        if constexpr (!std::is_same<K, hip_builtin_kernel>::value)
        {
            static_assert(hip_detail::user_kernels<K>::available,
                          "hip_sched::frames: a user kernel (a callable) is device code: include "
                          "visionaray_hip/hip_kernels.h and compile with hipcc");
            hip_detail::user_kernels<K>::frames(*ctx_, kernel, cams, rt, frame_num);
        }
        else
            frames_builtin(kernel, cams, rt, frame_num);
    }

private:
    template <typename Camera, typename RT>
    void frames_builtin(hip_builtin_kernel const& kernel, std::vector<Camera> const& cams, RT& rt, unsigned frame_num)
    {
        if (cams.empty() || rt.height() % cams.size() != 0)
            throw std::runtime_error("hip_sched::frames: render target height must be frames x image height");
        const uint32_t W = uint32_t(rt.width()), H = uint32_t(rt.height() / cams.size());
        std::vector<vrh_camera> c(cams.size());
        for (size_t f = 0; f < cams.size(); ++f)
        {
            auto const& cam = cams[f];
            float eye[3] = { cam.eye().x, cam.eye().y, cam.eye().z };
            float center[3] = { cam.center().x, cam.center().y, cam.center().z };
            float up[3] = { cam.up().x, cam.up().y, cam.up().z };
            hip_detail::check(vrh_make_camera(eye, center, up, cam.fovy(), cam.aspect(), W, H, &c[f]), "vrh_make_camera");
        }
        rt.begin_frame();
        hip_detail::check(vrh_render_batch(ctx_->get(), kernel.scene, rt.handle(), c.data(), uint32_t(c.size()),
                                           &kernel.desc, nullptr, frame_num),
                          "vrh_render_batch");
        rt.end_frame();
    }

public:
    hip_context& context() const { return *ctx_; }

private:
    std::shared_ptr<hip_context> ctx_;
    hip_render_group* group_ = nullptr;
    unsigned shards_ = 0;
};

// host-side builder with the reference's result (build<index_bvh<P>>, build.inl:165-178):
// fills nodes / indices of any container pair (resize(), data())
template <typename Primitive, typename NodeVec, typename IndexVec>
unsigned hip_build_index_bvh(Primitive const* prims, size_t n, NodeVec& nodes, IndexVec& indices)
{
    nodes.resize(2 * n);
    indices.resize(n);
    uint32_t nn = 0, depth = 0;
    hip_detail::check(vrh_build_bvh(prims, uint32_t(n),
                                    hip_detail::is_sphere<Primitive>::value ? VRH_PRIM_SPHERE48 : VRH_PRIM_TRI64,
                                    nodes.data(), &nn, indices.data(), &depth),
                      "vrh_build_bvh");
    nodes.resize(nn);
    return depth;
}

} // visionaray
