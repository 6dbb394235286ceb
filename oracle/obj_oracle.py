"""oracle/obj_oracle.py -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's OBJ loader.

Checker for libvrh's vrh_obj_load (visionaray_amd/csrc/vrh_obj.cpp).  Only tests/ may import it.

The reference parses OBJ with Boost.Spirit (src/common/obj_grammar.cpp:40-77) and builds its model in
load_obj (src/common/obj_loader.cpp:299-527).  Boost is absent from this image, so the reference
loader cannot be built here: PARITY UNPINNED against the reference binary.  This module restates it
independently of the C++ parser -- as PEG combinators composed exactly like the Spirit rules
(sequence / alternative / optional / kleene, the qi::blank skipper with pre-skip before every
primitive, rules declared without a skipper pre-skipping once on entry) and the model-building code
as straight-line Python over numpy float32 scalars -- and the tests pin both against each other and
against hand-derived expectations of the reference's documented behaviour.

Numbers: qi::float_ forms (significand digits accumulated in float) / (float power of ten); for at
most 7 significant digits and 10 fraction digits that is one correctly rounded division of exact
operands, i.e. the correctly rounded float of the decimal.  Here: float32(float(token)) (double, then
float), identical for such inputs (no 7-digit decimal lies within 2^-53 of a float midpoint).
"""
from __future__ import annotations

import math
import os

import numpy as np

F32 = np.float32

# ---- PEG combinators: parser(text, i, skip) -> (i', value) | None ------------------------------


def _skip(t, i):
    while i < len(t) and t[i] in " \t":
        i += 1
    return i


def lit(s):
    def p(t, i, sk):
        if sk:
            i = _skip(t, i)
        return (i + len(s), None) if t.startswith(s, i) else None
    return p


def eol(t, i, sk):
    if sk:
        i = _skip(t, i)
    if t.startswith("\r\n", i):
        return i + 2, None
    if i < len(t) and t[i] in "\r\n":
        return i + 1, None
    return None


def _digits(t, i):
    j = i
    while j < len(t) and t[j].isdigit() and t[j] in "0123456789":
        j += 1
    return j


def float_(t, i, sk):
    """qi::float_ (ureal_policies): [sign] (nan | inf[inity] | digits[.digits] | .digits) [exp]."""
    if sk:
        i = _skip(t, i)
    j = i
    sign = 1.0
    if j < len(t) and t[j] in "+-":
        sign = -1.0 if t[j] == "-" else 1.0
        j += 1
    low = t[j:j + 8].lower()
    if low.startswith("nan"):
        return j + 3, F32(math.copysign(math.nan, sign))
    if low.startswith("inf"):
        return j + (8 if low.startswith("infinity") else 3), F32(sign * math.inf)
    k = _digits(t, j)
    whole = k > j
    if k < len(t) and t[k] == ".":
        m = _digits(t, k + 1)
        if whole or m > k + 1:
            k = m
            whole = True
    if not whole:
        return None
    if k < len(t) and t[k] in "eE":
        m = k + 1
        if m < len(t) and t[m] in "+-":
            m += 1
        n = _digits(t, m)
        if n == m:
            return None                        # exponent prefix without digits: no match
        k = n
    return k, F32(sign * float(t[j:k]))


def int_(t, i, sk):
    if sk:
        i = _skip(t, i)
    j = i
    if j < len(t) and t[j] in "+-":
        j += 1
    k = _digits(t, j)
    if k == j:
        return None
    v = int(t[i:k])
    if not -2**31 <= v < 2**31:
        return None
    return k, v


def seq(*ps):
    def p(t, i, sk):
        out = []
        for q in ps:
            r = q(t, i, sk)
            if r is None:
                return None
            i, v = r
            if v is not None:
                out.append(v)
        return i, out
    return p


def alt(*ps):
    def p(t, i, sk):
        for q in ps:
            r = q(t, i, sk)
            if r is not None:
                return r
        return None
    return p


def opt(q, empty="none"):
    def p(t, i, sk):
        r = q(t, i, sk)
        return (i, empty) if r is None else r
    return p


def many(q):
    def p(t, i, sk):
        out = []
        while True:
            r = q(t, i, sk)
            if r is None:
                return i, out
            i, v = r
            out.append(v)
    return p


def text_to_eol(t, i, sk):                     # raw[*(char_ - eol)]
    j = i
    while j < len(t) and t[j] not in "\r\n":
        j += 1
    return j, t[i:j]


def rule(q, skipper):
    """qi::rule: a rule without skipper pre-skips once when invoked from a skipping context."""
    def p(t, i, sk):
        if sk and not skipper:
            i = _skip(t, i)
        return q(t, i, skipper)
    return p


# ---- the grammar, rule for rule (obj_grammar.cpp:40-77) ---------------------------------------

r_unhandled = rule(seq(text_to_eol, eol), False)
r_text_to_eol = rule(text_to_eol, False)
r_vec3 = rule(seq(float_, float_, float_), True)
r_newmtl = rule(seq(lit("newmtl"), r_text_to_eol, eol), True)
r_ka = rule(seq(lit("Ka"), r_vec3, eol), True)
r_kd = rule(seq(lit("Kd"), r_vec3, eol), True)
r_ke = rule(seq(lit("Ke"), r_vec3, eol), True)
r_ks = rule(seq(lit("Ks"), r_vec3, eol), True)
r_ns = rule(seq(lit("Ns"), float_, eol), True)
r_map_kd = rule(seq(lit("map_Kd"), r_text_to_eol, eol), True)
r_comment = rule(seq(lit("#"), r_text_to_eol, eol), False)
r_mtllib = rule(seq(lit("mtllib"), r_text_to_eol, eol), True)
r_usemtl = rule(seq(lit("usemtl"), r_text_to_eol, eol), True)
r_v = rule(alt(seq(lit("v"), float_, float_, float_, opt(float_), eol),
               seq(lit("v"), float_, float_, float_, float_, float_, float_, eol)), True)
r_vt = rule(seq(lit("vt"), float_, float_, opt(float_), eol), True)
r_vn = rule(seq(lit("vn"), r_vec3, eol), True)
r_vertices = rule(seq(r_v, many(r_v)), True)
r_tex_coords = rule(seq(r_vt, many(r_vt)), True)
r_normals = rule(seq(r_vn, many(r_vn)), True)
r_face_idx = rule(seq(int_, opt(lit("/"), None), opt(int_), opt(lit("/"), None), opt(int_)), False)
r_face = rule(seq(lit("f"), r_face_idx, r_face_idx, r_face_idx, many(r_face_idx), eol), True)


def _flat_vec(vals, n):
    return [v for v in vals[:n]]


# ---- model building (obj_loader.cpp) -----------------------------------------------------------

def default_material():
    """make_default_material (obj_loader.cpp:44-56) as a plastic record dict."""
    return dict(ca=[F32(0.2)] * 3, ka=F32(1), cd=[F32(0.8)] * 3, kd=F32(1), cs=[F32(0.1)] * 3, ks=F32(1),
                exp=F32(32))


def _cross(a, b):
    return [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]


def _dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def _remap(idx, size):                         # remap_index, obj_loader.cpp:58-62
    return size + idx if idx < 0 else idx - 1


class ObjError(ValueError):
    pass


def parse_mtl(path, lib):
    """parse_mtl (obj_loader.cpp:206-242); a final line without eol ends the file (the reference
    would loop forever there)."""
    t = open(path, "rb").read().decode("latin-1")
    i, cur = 0, None
    while i < len(t):
        r = r_newmtl(t, i, True)
        if r is not None:
            i, (name,) = r
            if name not in lib:
                lib[name] = dict(ka=[F32(0.2)] * 3, kd=[F32(0.8)] * 3, ke=[F32(0)] * 3, ks=[F32(0.1)] * 3,
                                 ns=F32(32), map_kd="")
            cur = lib[name]
            continue
        done = False
        if cur is not None:
            for key, rr in (("ka", r_ka), ("kd", r_kd), ("ke", r_ke), ("ks", r_ks)):
                # Spirit writes the attribute as it parses: a rule failing after some floats
                # leaves them behind
                partial = _partial_vec3(t, i, key)
                r = rr(t, i, True)
                if partial:
                    for k, v in enumerate(partial):
                        cur[key][k] = v
                if r is not None:
                    i, (vec,) = r
                    cur[key] = list(vec)
                    done = True
                    break
            if not done:
                r = r_ns(t, i, True)
                if r is None:
                    rp = seq(lit("Ns"), float_)(t, i, True)
                    if rp is not None:
                        cur["ns"] = rp[1][0]
                if r is not None:
                    i, (ns,) = r
                    cur["ns"] = ns
                    done = True
            if not done:
                r = r_map_kd(t, i, True)
                if r is not None:
                    i, (cur["map_kd"],) = r
                    done = True
        if done:
            continue
        r = r_unhandled(t, i, True)
        if r is None:
            break
        i = r[0]


def _partial_vec3(t, i, key):
    """floats a failing K? rule has already stored (Spirit writes attributes in place)."""
    kw = {"ka": "Ka", "kd": "Kd", "ke": "Ke", "ks": "Ks"}[key]
    r = lit(kw)(t, i, True)
    if r is None:
        return []
    j, out = r[0], []
    for _ in range(3):
        f = float_(t, j, True)
        if f is None:
            break
        j, v = f
        out.append(v)
    return out


def load_obj(filename):
    """load_obj (obj_loader.cpp:299-527) -> dict of numpy arrays in the C-ABI layouts."""
    t = open(filename, "rb").read().decode("latin-1")
    lib = {}
    verts, tcs, norms = [], [], []
    prims, sn, tc, mats, names, texs = [], [], [], [], [], []
    degenerate = unknown = missing = 0
    geom_id = 0
    i = 0
    while i < len(t):
        r = r_comment(t, i, True)
        if r is not None:
            i = r[0]
            continue
        r = r_mtllib(t, i, True)
        if r is not None:
            i, (name,) = r
            d = os.path.dirname(filename)                   # parent_path()
            path = d + "/" + name if d != "" or not filename.startswith("/") else "/" + name
            if os.path.exists(path):
                parse_mtl(path, lib)
            else:
                missing += 1
            continue
        r = r_usemtl(t, i, True)
        if r is not None:
            i, (name,) = r
            if name in lib:                                 # add_material, :248-262
                e = lib[name]
                mats.append(dict(ca=list(e["ka"]), ka=F32(1), cd=list(e["kd"]), kd=F32(1), cs=list(e["ks"]),
                                 ks=F32(1), exp=e["ns"]))
                names.append(name)
                texs.append(e["map_kd"])
            else:
                unknown += 1
            geom_id = 0 if not mats else len(mats) - 1
            continue
        r = r_vertices(t, i, True)
        if r is not None:
            i, (first, rest) = r
            for v in [first] + rest:
                verts.append(v[:3])
            continue
        r = r_tex_coords(t, i, True)
        if r is not None:
            i, (first, rest) = r
            for v in [first] + rest:
                tcs.append(v[:2])
            continue
        r = r_normals(t, i, True)
        if r is not None:
            i, (first, rest) = r
            for v in [first[0]] + [x[0] for x in rest]:
                norms.append(v)
            continue
        r = r_face(t, i, True)
        if r is not None:
            i, vals = r
            faces = vals[0:3] + vals[3]
            corners = []
            for f in faces:                                 # (v, t|None, n|None)
                vt = [x for x in f]
                corners.append((vt[0], vt[1] if vt[1] != "none" else None, vt[2] if vt[2] != "none" else None))
            nv = len(verts)
            for c in corners:
                k = _remap(c[0], nv)
                if not 0 <= k < nv:
                    raise ObjError(f"face vertex index {c[0]} out of range")
            i1 = _remap(corners[0][0], nv)
            for last in range(2, len(corners)):             # store_faces, :96-150
                a, b, c = corners[0], corners[last - 1], corners[last]
                v1 = verts[i1]
                e1 = [verts[_remap(b[0], nv)][k] - v1[k] for k in range(3)]
                e2 = [verts[_remap(c[0], nv)][k] - v1[k] for k in range(3)]
                cr = _cross(e1, e2)
                if np.sqrt(_dot(cr, cr)) == F32(0):         # store_triangle, :64-88
                    degenerate += 1
                    continue
                prims.append((0 if not mats else len(mats) - 1, len(prims), list(v1), e1, e2))
                if a[1] is not None and b[1] is not None and c[1] is not None:
                    for x in (a, b, c):
                        k = _remap(x[1], len(tcs))
                        if not 0 <= k < len(tcs):
                            raise ObjError("tex coord index out of range")
                        tc.append(tcs[k])
                if a[2] is not None and b[2] is not None and c[2] is not None:
                    for x in (a, b, c):
                        k = _remap(x[2], len(norms))
                        if not 0 <= k < len(norms):
                            raise ObjError("normal index out of range")
                        sn.append(norms[k])
            continue
        r = r_unhandled(t, i, True)
        if r is None:
            break                                           # ++it over a final line without eol
        i = r[0]

    out = {}
    P = np.zeros(len(prims), [("geom_id", "<u4"), ("prim_id", "<u4"), ("pad", "<u4", 2), ("v1", "<f4", 4),
                              ("e1", "<f4", 4), ("e2", "<f4", 4)])
    gn = np.zeros((len(prims), 4), np.float32)
    lo = [F32(np.finfo(np.float32).max)] * 3
    hi = [F32(-np.finfo(np.float32).max)] * 3
    for k, (g, pid, v1, e1, e2) in enumerate(prims):
        P[k]["geom_id"], P[k]["prim_id"] = g, pid
        P[k]["v1"][:3], P[k]["e1"][:3], P[k]["e2"][:3] = v1, e1, e2
        cr = _cross(e1, e2)
        inv = F32(1) / np.sqrt(_dot(cr, cr))               # normalize = v * rsqrt(dot(v, v))
        gn[k, :3] = [cr[0] * inv, cr[1] * inv, cr[2] * inv]
        for p in (v1, [v1[j] + e1[j] for j in range(3)], [v1[j] + e2[j] for j in range(3)]):
            lo = [lo[j] if lo[j] < p[j] else p[j] for j in range(3)]
            hi = [p[j] if hi[j] < p[j] else hi[j] for j in range(3)]
    i = len(tc)                                             # dummy tex coords, :504-510
    while i < len(prims):
        tc += [[F32(0), F32(0)]] * 3
        i += 1
    for _ in range(len(mats), geom_id + 1):                 # :512-516
        mats.append(default_material())
        names.append("")
        texs.append("")
    M = np.zeros(len(mats), [("ca", "<f4", 3), ("ka", "<f4"), ("cd", "<f4", 3), ("kd", "<f4"), ("cs", "<f4", 3),
                             ("ks", "<f4"), ("exp", "<f4")])
    for k, m in enumerate(mats):
        for f in ("ca", "ka", "cd", "kd", "cs", "ks", "exp"):
            M[k][f] = m[f]
    out["primitives"] = P
    out["geometric_normals"] = gn
    out["shading_normals"] = np.array([[n[0], n[1], n[2], 0] for n in sn], np.float32).reshape(-1, 4)
    out["tex_coords"] = np.array(tc, np.float32).reshape(-1, 2)
    out["materials"] = M
    out["material_names"] = names
    out["textures"] = texs
    out["bbox"] = np.array([lo, hi], np.float32)
    out["num_degenerate"], out["num_unknown_materials"], out["num_missing_files"] = degenerate, unknown, missing
    return out
