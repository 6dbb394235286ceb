// visionaray_amd/csrc/vrh_obj.cpp -- Wavefront OBJ / MTL input.
//
// Restates load_obj (src/common/obj_loader.cpp:299-527) and its Boost.Spirit grammar
// (obj_grammar.cpp:40-77) as a hand-written recursive-descent parser, so real models can feed the
// traversal without Boost.  The model it produces is the reference's `model` (model.h:20-49):
//   * primitives: one basic_triangle per fan triangle of every face (store_faces, :96-150), ids
//     assigned by store_triangle (:64-88): prim_id = number of triangles kept so far, geom_id =
//     index of the last material added by `usemtl` (0 before any); zero-area triangles
//     (length(cross(e1, e2)) == 0) are dropped and consume no prim_id;
//   * shading_normals / tex_coords: three per kept triangle whose three corners all carry a vn / vt
//     index; tex_coords then padded by the reference's dummy loop (:504-510);
//   * geometric_normals: normalize(cross(e1, e2)) per triangle (:497-502);
//   * materials: plastic<float> per successful `usemtl` (add_material, :248-262: ca = Ka, cd = Kd,
//     cs = Ks, ka = kd = ks = 1, exp = Ns; MTL defaults from make_default_material, :44-56), padded
//     with default materials up to the last geom_id (:512-516);
//   * bbox: combine() over v1, v1 + e1, v1 + e2 of every triangle (bounds, :156-174).
//
// The parser walks the same rules in the same order as load_obj's loop (:331-492): comment,
// mtllib, usemtl, v, vt, vn, f, otherwise skip the line.  Grammar consequences kept on purpose:
// keywords need no blank after them ("v1 2 3" is a vertex), a face corner is int[/[int][/[int]]]
// with no blanks inside, `v` takes 3 or 4 numbers (w ignored) or 6 (colour extension, ignored),
// names run to the end of the line (trailing blanks included), negative indices count back from
// the vertices read so far (remap_index, :58-62), and a last line without an end-of-line is
// ignored (every rule ends in qi::eol).  Where the reference is undefined (face index 0 or out of
// range) this loader fails with VRH_ERR_INVALID instead; a missing mtllib is a warning, as there.
//
// Numbers: qi::float_ accumulates the significand digits in float and divides by a float power of
// ten; for inputs with at most 7 significant digits and 10 fraction digits both operands are exact
// and that single division is correctly rounded, i.e. identical to std::from_chars used here.
// Longer inputs can differ in the last bit from Boost's result (parity unpinned there; Boost is
// absent from this image).  Arithmetic on the parsed values is float, -ffp-contract=off.
#include "vrh_internal.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <map>
#include <string>
#include <sys/stat.h>
#include <vector>

using namespace vrh;

namespace {

struct v3 { float x, y, z; };
inline v3 sub(v3 a, v3 b) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
inline v3 add(v3 a, v3 b) { return { a.x + b.x, a.y + b.y, a.z + b.z }; }
inline v3 cross(v3 a, v3 b) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float vmin(float x, float y) { return x < y ? x : y; }      // math.h:48-60
inline float vmax(float x, float y) { return x < y ? y : x; }

struct face_index { int v; bool has_t, has_n; int t, n; };

// material as parsed from an MTL file (struct mtl, obj_loader.cpp:180-200)
struct mtl_entry
{
    v3 ka{ 0.2f, 0.2f, 0.2f }, kd{ 0.8f, 0.8f, 0.8f }, ke{ 0.0f, 0.0f, 0.0f }, ks{ 0.1f, 0.1f, 0.1f };
    float ns = 32.0f;
    std::string map_kd;
};

vrh_plastic default_material()                                  // make_default_material, :44-56
{
    vrh_plastic m;
    m.ca[0] = m.ca[1] = m.ca[2] = 0.2f; m.ka = 1.0f;
    m.cd[0] = m.cd[1] = m.cd[2] = 0.8f; m.kd = 1.0f;
    m.cs[0] = m.cs[1] = m.cs[2] = 0.1f; m.ks = 1.0f;
    m.exp = 32.0f;
    return m;
}

// ---- lexical primitives of the grammar (qi::blank skipper, qi::eol, qi::float_, qi::int_) -----

struct cursor
{
    const char* p;
    const char* end;
    bool at_end() const { return p == end; }
    void skip_blank() { while (p != end && (*p == ' ' || *p == '\t')) ++p; }
    bool lit(const char* s)                                    // literal, after pre-skip
    {
        skip_blank();
        const char* q = p;
        for (; *s; ++s, ++q)
            if (q == end || *q != *s) return false;
        p = q;
        return true;
    }
    bool eol()                                                  // "\r\n" | '\r' | '\n', after pre-skip
    {
        skip_blank();
        if (p == end) return false;
        if (*p == '\r') { ++p; if (p != end && *p == '\n') ++p; return true; }
        if (*p == '\n') { ++p; return true; }
        return false;
    }
    // raw[*(char_ - eol)]: the rest of the line, pre-skipped
    std::string text_to_eol()
    {
        skip_blank();
        const char* q = p;
        while (q != end && *q != '\r' && *q != '\n') ++q;
        std::string s(p, q);
        p = q;
        return s;
    }
    bool number(float& out)                                      // qi::float_, after pre-skip
    {
        skip_blank();
        const char* q = p;
        bool neg = false;
        if (q != end && (*q == '+' || *q == '-')) { neg = *q == '-'; ++q; }
        const char* s = q;                                      // unsigned part
        auto ci_lit = [&](const char* w) {
            const char* r = q;
            for (; *w; ++w, ++r)
                if (r == end || (*r | 0x20) != *w) return (const char*)nullptr;
            return r;
        };
        if (const char* r = ci_lit("nan"))
        {
            out = neg ? -std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::quiet_NaN();
            p = r;
            return true;
        }
        if (const char* r = ci_lit("inf"))
        {
            q = r;
            if (const char* r2 = ci_lit("inity")) q = r2;
            out = neg ? -std::numeric_limits<float>::infinity() : std::numeric_limits<float>::infinity();
            p = q;
            return true;
        }
        bool digits = false;
        while (q != end && *q >= '0' && *q <= '9') { ++q; digits = true; }
        if (q != end && *q == '.')
        {
            const char* r = q + 1;
            bool frac = false;
            while (r != end && *r >= '0' && *r <= '9') { ++r; frac = true; }
            if (digits || frac) { q = r; digits = true; }
        }
        if (!digits) return false;
        if (q != end && (*q == 'e' || *q == 'E'))
        {
            const char* r = q + 1;
            if (r != end && (*r == '+' || *r == '-')) ++r;
            if (r == end || *r < '0' || *r > '9') return false;   // exponent prefix without digits: no match
            while (r != end && *r >= '0' && *r <= '9') ++r;
            q = r;
        }
        float v = 0.0f;
        if (fast_decimal(s, q, v))
        {
            out = neg ? -v : v;
            p = q;
            return true;
        }
        auto res = std::from_chars(s, q, v, std::chars_format::general);
        if (res.ec == std::errc::result_out_of_range)
        {
            // from_chars leaves v untouched on range errors: overflow -> inf, underflow -> 0
            const double d = std::strtod(std::string(s, q).c_str(), nullptr);
            v = static_cast<float>(d);
        }
        else if (res.ec != std::errc() || res.ptr != q)
            return false;
        out = neg ? -v : v;
        p = q;
        return true;
    }
    // Clinger's fast path in float: significand w <= 2^24 and |10-exponent| <= 10 make w and 10^k
    // exact floats, so one multiply / divide is the correctly rounded result (and qi::float_'s)
    static bool fast_decimal(const char* s, const char* q, float& out)
    {
        static const float p10[11] = { 1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f };
        uint32_t w = 0;
        int e10 = 0;
        const char* r = s;
        for (; r != q && *r >= '0' && *r <= '9'; ++r)
        {
            w = w * 10u + uint32_t(*r - '0');
            if (w > (1u << 24)) return false;
        }
        if (r != q && *r == '.')
            for (++r; r != q && *r >= '0' && *r <= '9'; ++r)
            {
                w = w * 10u + uint32_t(*r - '0');
                if (w > (1u << 24)) return false;
                --e10;
            }
        if (r != q)                                              // exponent
        {
            ++r;
            bool eneg = false;
            if (*r == '+' || *r == '-') { eneg = *r == '-'; ++r; }
            int e = 0;
            for (; r != q; ++r)
            {
                e = e * 10 + (*r - '0');
                if (e > 100) return false;
            }
            e10 += eneg ? -e : e;
        }
        if (e10 < -10 || e10 > 10) return false;
        const float fw = static_cast<float>(w);
        out = e10 >= 0 ? fw * p10[e10] : fw / p10[-e10];
        return true;
    }
    bool integer(int& out)                                       // qi::int_, no pre-skip
    {
        const char* q = p;
        bool neg = false;
        if (q != end && (*q == '+' || *q == '-')) { neg = *q == '-'; ++q; }
        if (q == end || *q < '0' || *q > '9') return false;
        long long v = 0;
        while (q != end && *q >= '0' && *q <= '9')
        {
            v = v * 10 + (*q - '0');
            if (v > 2147483648LL) return false;                  // overflow fails the parse
            ++q;
        }
        if (neg) v = -v;
        if (v > 2147483647LL) return false;
        out = static_cast<int>(v);
        p = q;
        return true;
    }
    // r_face_idx (obj_grammar.cpp:71): int_ >> -'/' >> -int_ >> -'/' >> -int_, no skipper inside
    bool face_idx(face_index& f)
    {
        skip_blank();
        f = face_index{ 0, false, false, 0, 0 };
        if (!integer(f.v)) return false;
        if (p != end && *p == '/') ++p;
        if (integer(f.t)) f.has_t = true;
        if (p != end && *p == '/') ++p;
        if (integer(f.n)) f.has_n = true;
        return true;
    }
};

bool file_exists(const std::string& path)
{
    struct stat st;
    return ::stat(path.c_str(), &st) == 0;
}

bool read_file(const std::string& path, std::string& out)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    struct stat st;
    if (::fstat(fileno(f), &st) != 0 || !S_ISREG(st.st_mode)) { std::fclose(f); return false; }
    out.resize(static_cast<size_t>(st.st_size));
    const size_t got = out.empty() ? 0 : std::fread(&out[0], 1, out.size(), f);
    std::fclose(f);
    return got == out.size();
}

// boost::filesystem::path(filename).parent_path().string() + "/" + name (obj_loader.cpp:343-345)
std::string sibling(const std::string& filename, const std::string& name)
{
    const size_t slash = filename.find_last_of('/');
    std::string dir = slash == std::string::npos ? std::string() : filename.substr(0, slash);
    if (slash == 0) dir = "/";
    return dir + "/" + name;
}

// three floats into a vec3 attribute, written as they parse (a failing rule leaves a prefix)
bool vec3_into(cursor& c, v3& v)
{
    return c.number(v.x) && c.number(v.y) && c.number(v.z);
}

// parse_mtl (obj_loader.cpp:206-242)
bool parse_mtl(const std::string& path, std::map<std::string, mtl_entry>& lib, std::string& err)
{
    std::string text;
    if (!read_file(path, text)) { err = "cannot read mtllib " + path; return false; }
    cursor c{ text.data(), text.data() + text.size() };
    mtl_entry* cur = nullptr;
    while (!c.at_end())
    {
        cursor t = c;
        if (t.lit("newmtl"))
        {
            std::string name = t.text_to_eol();
            if (t.eol())
            {
                cur = &lib.emplace(name, mtl_entry{}).first->second;   // existing entry kept as is
                c = t;
                continue;
            }
        }
        struct { const char* kw; v3 mtl_entry::* field; } vecs[] = {
            { "Ka", &mtl_entry::ka }, { "Kd", &mtl_entry::kd }, { "Ke", &mtl_entry::ke }, { "Ks", &mtl_entry::ks } };
        bool done = false;
        if (cur)
        {
            for (auto& r : vecs)
            {
                t = c;
                if (t.lit(r.kw) && vec3_into(t, cur->*r.field) && t.eol()) { c = t; done = true; break; }
            }
            if (!done)
            {
                t = c;
                if (t.lit("Ns") && t.number(cur->ns) && t.eol()) { c = t; done = true; }
            }
            if (!done)
            {
                t = c;
                if (t.lit("map_Kd"))
                {
                    std::string s = t.text_to_eol();
                    if (t.eol()) { cur->map_kd = s; c = t; done = true; }
                }
            }
        }
        if (done) continue;
        // r_unhandled; the reference loops forever on a final line without eol -- stop there
        t = c;
        t.skip_blank();
        while (!t.at_end() && *t.p != '\r' && *t.p != '\n') ++t.p;
        if (!t.eol()) break;
        c = t;
    }
    return true;
}

struct obj_model
{
    std::vector<tri64> primitives;
    std::vector<v3> shading_normals, geometric_normals;
    std::vector<float> tex_coords;          // 2 per entry
    std::vector<vrh_plastic> materials;
    std::vector<std::string> material_names, textures;   // per material: usemtl name, map_Kd
    v3 bbox_min, bbox_max;
    uint32_t degenerate = 0, unknown_materials = 0, missing_files = 0;
};

int remap(int idx, int size) { return idx < 0 ? size + idx : idx - 1; }   // remap_index, :58-62

// store_triangle (:64-88)
bool store_triangle(obj_model& m, const std::vector<v3>& verts, int i1, int i2, int i3)
{
    const v3 v1 = verts[i1];
    const v3 e1 = sub(verts[i2], v1), e2 = sub(verts[i3], v1);
    const v3 n = cross(e1, e2);
    if (std::sqrt(dot(n, n)) == 0.0f) { ++m.degenerate; return false; }
    tri64 t{};
    t.prim_id = static_cast<uint32_t>(m.primitives.size());
    t.geom_id = m.materials.empty() ? 0u : static_cast<uint32_t>(m.materials.size() - 1);
    t.v1[0] = v1.x; t.v1[1] = v1.y; t.v1[2] = v1.z;
    t.e1[0] = e1.x; t.e1[1] = e1.y; t.e1[2] = e1.z;
    t.e2[0] = e2.x; t.e2[1] = e2.y; t.e2[2] = e2.z;
    m.primitives.push_back(t);
    return true;
}

// store_faces (:96-150): triangle fan around the first corner
bool store_faces(obj_model& m, const std::vector<v3>& verts, const std::vector<float>& tcs,
                 const std::vector<v3>& norms, const std::vector<face_index>& f, std::string& err)
{
    const int nv = static_cast<int>(verts.size());
    const int nt = static_cast<int>(tcs.size() / 2);
    const int nn = static_cast<int>(norms.size());
    auto bad = [&](const char* what, int idx, int size) {
        err = std::string("face ") + what + " index " + std::to_string(idx) + " out of range (" +
              std::to_string(size) + " defined)";
        return false;
    };
    for (const auto& c : f)
    {
        const int i = remap(c.v, nv);
        if (i < 0 || i >= nv) return bad("vertex", c.v, nv);
    }
    const int i1 = remap(f[0].v, nv);
    for (size_t last = 2; last != f.size(); ++last)
    {
        const face_index& a = f[0];
        const face_index& b = f[last - 1];
        const face_index& c = f[last];
        if (!store_triangle(m, verts, i1, remap(b.v, nv), remap(c.v, nv))) continue;
        if (a.has_t && b.has_t && c.has_t)
        {
            for (const face_index* x : { &a, &b, &c })
            {
                const int ti = remap(x->t, nt);
                if (ti < 0 || ti >= nt) return bad("tex coord", x->t, nt);
                m.tex_coords.push_back(tcs[2 * ti]);
                m.tex_coords.push_back(tcs[2 * ti + 1]);
            }
        }
        if (a.has_n && b.has_n && c.has_n)
        {
            for (const face_index* x : { &a, &b, &c })
            {
                const int ni = remap(x->n, nn);
                if (ni < 0 || ni >= nn) return bad("normal", x->n, nn);
                m.shading_normals.push_back(norms[ni]);
            }
        }
    }
    return true;
}

int load_obj(const std::string& filename, obj_model& m, std::string& err)
{
    std::string text;
    if (!read_file(filename, text)) { err = "cannot read " + filename; return VRH_ERR_INVALID; }
    std::map<std::string, mtl_entry> lib;
    size_t geom_id = 0;
    std::vector<v3> verts, norms;
    std::vector<float> tcs;
    std::vector<face_index> faces;
    cursor c{ text.data(), text.data() + text.size() };
    while (!c.at_end())
    {
        cursor t = c;
        if (t.lit("#"))                                            // r_comment
        {
            t.text_to_eol();
            if (t.eol()) { c = t; continue; }
        }
        t = c;
        if (t.lit("mtllib"))
        {
            const std::string name = t.text_to_eol();
            if (t.eol())
            {
                c = t;
                const std::string path = sibling(filename, name);
                if (file_exists(path))
                {
                    if (!parse_mtl(path, lib, err)) return VRH_ERR_INVALID;
                }
                else
                {
                    ++m.missing_files;
                    std::fprintf(stderr, "Warning: file does not exist: %s\n", path.c_str());
                }
                continue;
            }
        }
        t = c;
        if (t.lit("usemtl"))
        {
            const std::string name = t.text_to_eol();
            if (t.eol())
            {
                c = t;
                auto it = lib.find(name);
                if (it != lib.end())
                {
                    const mtl_entry& e = it->second;                // add_material, :248-262
                    vrh_plastic p;
                    p.ca[0] = e.ka.x; p.ca[1] = e.ka.y; p.ca[2] = e.ka.z; p.ka = 1.0f;
                    p.cd[0] = e.kd.x; p.cd[1] = e.kd.y; p.cd[2] = e.kd.z; p.kd = 1.0f;
                    p.cs[0] = e.ks.x; p.cs[1] = e.ks.y; p.cs[2] = e.ks.z; p.ks = 1.0f;
                    p.exp = e.ns;
                    m.materials.push_back(p);
                    m.material_names.push_back(name);
                    m.textures.push_back(e.map_kd);
                }
                else
                {
                    ++m.unknown_materials;
                    std::fprintf(stderr, "Warning: material not present in mtllib: %s\n", name.c_str());
                }
                geom_id = m.materials.empty() ? 0 : m.materials.size() - 1;
                continue;
            }
        }
        // r_vertices: ("v" 3 floats [float] eol | "v" 6 floats eol)+, xyz kept
        {
            bool any = false;
            for (;;)
            {
                t = c;
                v3 v{};
                bool ok = false;
                if (t.lit("v") && vec3_into(t, v))
                {
                    cursor u = t;
                    float w;
                    if (u.number(w)) { if (u.eol()) { t = u; ok = true; } }   // x y z w
                    else if (u.eol()) { t = u; ok = true; }                  // x y z
                    if (!ok)                                                  // x y z r g b
                    {
                        u = t;
                        float r, g, b;
                        if (u.number(r) && u.number(g) && u.number(b) && u.eol()) { t = u; ok = true; }
                    }
                }
                if (!ok) break;
                verts.push_back(v);
                c = t;
                any = true;
            }
            if (any) continue;
        }
        // r_tex_coords: ("vt" float float [float] eol)+
        {
            bool any = false;
            for (;;)
            {
                t = c;
                float s, tt, w;
                bool ok = false;
                if (t.lit("vt") && t.number(s) && t.number(tt))
                {
                    cursor u = t;
                    if (u.number(w) && u.eol()) { t = u; ok = true; }
                    else if (t.eol()) ok = true;
                }
                if (!ok) break;
                tcs.push_back(s);
                tcs.push_back(tt);
                c = t;
                any = true;
            }
            if (any) continue;
        }
        // r_normals: ("vn" vec3 eol)+
        {
            bool any = false;
            for (;;)
            {
                t = c;
                v3 n{};
                if (!(t.lit("vn") && vec3_into(t, n) && t.eol())) break;
                norms.push_back(n);
                c = t;
                any = true;
            }
            if (any) continue;
        }
        // r_face: "f" idx idx idx idx* eol
        t = c;
        faces.clear();
        if (t.lit("f"))
        {
            face_index fi;
            while (t.face_idx(fi)) faces.push_back(fi);
            if (faces.size() >= 3 && t.eol())
            {
                c = t;
                if (!store_faces(m, verts, tcs, norms, faces, err)) return VRH_ERR_INVALID;
                continue;
            }
        }
        // r_unhandled, else ++it: a final line without eol matches nothing and is skipped
        t = c;
        t.skip_blank();
        while (!t.at_end() && *t.p != '\r' && *t.p != '\n') ++t.p;
        if (!t.eol()) break;
        c = t;
    }
    // geometric normals (:497-502): normalize = v * rsqrt(dot(v, v)) (vector3.inl:333-336)
    m.geometric_normals.reserve(m.primitives.size());
    for (const tri64& t : m.primitives)
    {
        const v3 n = cross(v3{ t.e1[0], t.e1[1], t.e1[2] }, v3{ t.e2[0], t.e2[1], t.e2[2] });
        const float inv = 1.0f / std::sqrt(dot(n, n));
        m.geometric_normals.push_back(v3{ n.x * inv, n.y * inv, n.z * inv });
    }
    // dummy tex coords (:504-510): three per iteration, counter compared against the triangle count
    for (size_t i = m.tex_coords.size() / 2; i < m.primitives.size(); ++i)
        m.tex_coords.insert(m.tex_coords.end(), 6, 0.0f);
    // a material for each geometry (:512-516)
    for (size_t i = m.materials.size(); i <= geom_id; ++i)
    {
        m.materials.push_back(default_material());
        m.material_names.emplace_back();
        m.textures.emplace_back();
    }
    // bounds (:156-174)
    v3 lo{ std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max() };
    v3 hi{ std::numeric_limits<float>::lowest(), std::numeric_limits<float>::lowest(), std::numeric_limits<float>::lowest() };
    for (const tri64& t : m.primitives)
    {
        const v3 a{ t.v1[0], t.v1[1], t.v1[2] };
        const v3 pts[3] = { a, add(a, v3{ t.e1[0], t.e1[1], t.e1[2] }), add(a, v3{ t.e2[0], t.e2[1], t.e2[2] }) };
        for (const v3& p : pts)
        {
            lo = v3{ vmin(lo.x, p.x), vmin(lo.y, p.y), vmin(lo.z, p.z) };
            hi = v3{ vmax(hi.x, p.x), vmax(hi.y, p.y), vmax(hi.z, p.z) };
        }
    }
    m.bbox_min = lo;
    m.bbox_max = hi;
    return VRH_OK;
}

} // namespace

struct vrh_obj : obj_model {};

extern "C" VRH_API int vrh_obj_load(const char* filename, vrh_obj** out)
{
    if (!filename || !out) { set_error("vrh_obj_load: null argument"); return VRH_ERR_INVALID; }
    *out = nullptr;
    try
    {
        auto m = new vrh_obj();
        std::string err;
        const int rc = load_obj(filename, *m, err);
        if (rc != VRH_OK)
        {
            delete m;
            set_error("vrh_obj_load: " + err);
            return rc;
        }
        *out = m;
        return VRH_OK;
    }
    catch (const std::bad_alloc&)
    {
        set_error("vrh_obj_load: out of host memory");
        return VRH_ERR_OOM;
    }
}

extern "C" VRH_API int vrh_obj_get_info(const vrh_obj* m, vrh_obj_info* info)
{
    if (!m || !info) { set_error("vrh_obj_get_info: null argument"); return VRH_ERR_INVALID; }
    std::memset(info, 0, sizeof(*info));
    info->num_triangles = static_cast<uint32_t>(m->primitives.size());
    info->num_shading_normals = static_cast<uint32_t>(m->shading_normals.size());
    info->num_tex_coords = static_cast<uint32_t>(m->tex_coords.size() / 2);
    info->num_materials = static_cast<uint32_t>(m->materials.size());
    info->num_degenerate = m->degenerate;
    info->num_unknown_materials = m->unknown_materials;
    info->num_missing_files = m->missing_files;
    info->bbox_min[0] = m->bbox_min.x; info->bbox_min[1] = m->bbox_min.y; info->bbox_min[2] = m->bbox_min.z;
    info->bbox_max[0] = m->bbox_max.x; info->bbox_max[1] = m->bbox_max.y; info->bbox_max[2] = m->bbox_max.z;
    return VRH_OK;
}

extern "C" VRH_API int vrh_obj_get_data(const vrh_obj* m, void* triangles, float* geometric_normals,
                                        float* shading_normals, float* tex_coords, vrh_plastic* materials)
{
    if (!m) { set_error("vrh_obj_get_data: null model"); return VRH_ERR_INVALID; }
    if (triangles && !m->primitives.empty())
        std::memcpy(triangles, m->primitives.data(), m->primitives.size() * sizeof(tri64));
    auto put4 = [](float* out, const std::vector<v3>& v) {
        for (size_t i = 0; i < v.size(); ++i)
        {
            out[4 * i] = v[i].x; out[4 * i + 1] = v[i].y; out[4 * i + 2] = v[i].z; out[4 * i + 3] = 0.0f;
        }
    };
    if (geometric_normals) put4(geometric_normals, m->geometric_normals);
    if (shading_normals) put4(shading_normals, m->shading_normals);
    if (tex_coords && !m->tex_coords.empty())
        std::memcpy(tex_coords, m->tex_coords.data(), m->tex_coords.size() * sizeof(float));
    if (materials && !m->materials.empty())
        std::memcpy(materials, m->materials.data(), m->materials.size() * sizeof(vrh_plastic));
    return VRH_OK;
}

extern "C" VRH_API const char* vrh_obj_material_name(const vrh_obj* m, uint32_t index)
{
    if (!m || index >= m->material_names.size()) return nullptr;
    return m->material_names[index].c_str();
}

extern "C" VRH_API const char* vrh_obj_material_texture(const vrh_obj* m, uint32_t index)
{
    if (!m || index >= m->textures.size()) return nullptr;
    return m->textures[index].c_str();
}

extern "C" VRH_API int vrh_obj_free(vrh_obj* m)
{
    delete m;
    return VRH_OK;
}
