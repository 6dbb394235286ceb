"""CPU: the float identity the whitted kernel's LDS surface relies on (vrh_shade.h whitted_reflect).

The kernel keeps only the two-sided shading normal n = faceforward(sn) = +-sn of a bounce and
recomputes the reflection reflect(view, sn) = 2 * dot(sn, view) * sn - view (vector.inl:683-689,
whitted.inl:262) from n.  Under round-to-nearest negation commutes with every product and sum, so
the result is bit-identical whichever sign n carries; checked here in float32 with the kernel's
operation order (no FMA) over random and edge-case vectors.
"""
import numpy as np

f32 = np.float32


def dot(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def reflect(n, v):
    d2 = f32(f32(2.0) * dot(n, v))
    return np.array([f32(f32(d2 * n[0]) - v[0]), f32(f32(d2 * n[1]) - v[1]), f32(f32(d2 * n[2]) - v[2])], np.float32)


def test_reflect_is_sign_invariant_bitwise():
    rng = np.random.default_rng(7)
    vecs = rng.standard_normal((20000, 2, 3)).astype(np.float32)
    vecs[:100] *= f32(1e-30)                          # tiny values (subnormal products)
    vecs[100:200] *= f32(1e18)                        # huge values
    vecs[200:300, :, 1] = 0.0                         # signed zeros
    vecs[300:400, 0] = -vecs[300:400, 1]              # anti-parallel normal / view
    with np.errstate(over="ignore", under="ignore", invalid="ignore"):
        for sn, v in vecs:
            a, b = reflect(sn, v), reflect(-sn, v)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) or (np.isnan(a).all() and np.isnan(b).all())
