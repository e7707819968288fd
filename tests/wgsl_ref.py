"""Independent per-pixel restatement of the reference's live pipeline, straight from the WGSL.

Test infrastructure only (the checker of the C oracle, tests/test_wgsl_ref.py): PT_01
(G-buffer), PT_1 (initial path-tree RIS, one reservoir per pixel) and PT_4 (final shading +
accumulation) for single pixels, written from the shader sources function by function --
NOT from oracle/pt_oracle.c.  SH/ = apps/frontend/src/graphics-core/shaders/ in the reference.

What is deliberately different from the oracle (so a shared misreading does not pass):
  * it reads the reference buffers exactly as the shaders do (GetInstance, GetMeshDescriptor,
    GetBlasNode with the 8-word BlasNode records, GetTriangle through the index buffer) -- the
    oracle and the HIP kernels walk a derived node-pair layout;
  * TraceRay runs the WGSL loop literally: every instance, every sub-mesh root, the 64-entry
    stack, the full [1e-4, 1e10] range even for Visibility (the fast paths cap at the light);
  * Visibility, SampleNEE's CDF search, UpdateReservoir, CompressPath / SafeReconnectionIndex,
    RegeneratePath, PathContribution and WriteColor are restated as written, including the
    quirks that fall out of the code (a path snapshot's Lobe[i] is still 0 at vertex i's NEE,
    PathTree.rSeed[i + 1] is overwritten by the BSDF seed, PT_4's PDF_LIGHT / L_emit without
    the EPS clamps, the G-buffer pass's own epsilons).

What is shared by construction (the implementation-defined WGSL points DESIGN.md §2 fixes for
every implementation): f32 arithmetic with left-to-right sums and no FMA (numpy float32 scalars,
one rounding per operation), normalize = v / length(v), mix(a, b, t) = a (1 - t) + b t, min /
max = IEEE minNum / maxNum, correctly rounded / and sqrt, pow(x, 5) = (x^2)^2 x and the fixed
Cody-Waite + minimax sin / cos (restated below from their definition), reflect / refract as
the WGSL spec writes them, out-of-range array reads clamped (WGSL robustness).
"""
from __future__ import annotations

from collections import Counter

import numpy as np

f32 = np.float32
Z = f32(0.0)
ONE = f32(1.0)
INF = f32(1e11)
EPS = f32(1e-4)
PI = f32(3.141592)
ENV = (f32(0.5), f32(0.5), f32(0.5))
LIGHT_DIRECTION, LIGHT_POINT, LIGHT_RECT, LIGHT_ENV = 0, 1, 2, 3
LOBE_LAMBERT, LOBE_GGX, LOBE_NEE, LOBE_LIGHT = 0, 1, 2, 3
STRIDE_INSTANCE, STRIDE_LIGHT, STRIDE_DESCRIPTOR, STRIDE_MATERIAL, STRIDE_VERTEX, STRIDE_BLAS = 33, 18, 6, 15, 8, 8
U32 = 0xFFFFFFFF
# branch coverage of the restated code over a test's pixels (tests/test_wgsl_ref.py asserts
# that the bit-exact comparison went through each of these)
STATS = Counter()

# ------------------------------------------------------------------ f32 vector algebra (tuples)


def vadd(a, b):
    return (a[0] + b[0], a[1] + b[1], a[2] + b[2])


def vsub(a, b):
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def vmul(a, b):
    return (a[0] * b[0], a[1] * b[1], a[2] * b[2])


def vscale(a, s):
    return (a[0] * s, a[1] * s, a[2] * s)


def sscale(s, a):  # s * vec (WGSL scalar * vector: s * a_i)
    return (s * a[0], s * a[1], s * a[2])


def vdivs(a, s):
    return (a[0] / s, a[1] / s, a[2] / s)


def vneg(a):
    return (-a[0], -a[1], -a[2])


def dot(a, b):
    return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]


def cross(a, b):
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def length(a):
    return np.sqrt(dot(a, a))


def normalize(a):
    return vdivs(a, length(a))


def fmin(a, b):
    return np.fmin(a, b)


def fmax(a, b):
    return np.fmax(a, b)


def saturate(x):
    return fmin(fmax(x, Z), ONE)


def mix(a, b, t):
    return a * (ONE - t) + b * t


def vmix(a, b, t):
    return (mix(a[0], b[0], t), mix(a[1], b[1], t), mix(a[2], b[2], t))


def reflect(e1, e2):
    """WGSL reflect(e1, e2) = e1 - 2 * dot(e2, e1) * e2."""
    return vsub(e1, sscale(f32(2.0) * dot(e2, e1), e2))


def refract(e1, e2, e3):
    """WGSL refract: k = 1 - e3 e3 (1 - dot(e2, e1)^2); 0 if k < 0, else e3 e1 - (e3 dot + sqrt k) e2."""
    d = dot(e2, e1)
    k = ONE - e3 * e3 * (ONE - d * d)
    if k < Z:
        return (Z, Z, Z)
    return vsub(sscale(e3, e1), sscale(e3 * d + np.sqrt(k), e2))


def pow5(x):
    x2 = x * x
    return (x2 * x2) * x


def sincos(x):
    """The fixed f32 sin / cos every implementation here uses: reduction by pi/4
    in three Cody-Waite parts, then the single-precision minimax polynomials; x >= 0."""
    j = int(x * f32(1.27323954473516))
    y = f32(j)
    if j & 1:
        j += 1
        y = y + ONE
    j &= 7
    z = ((x - y * f32(0.78515625)) - y * f32(2.4187564849853515625e-4)) - y * f32(3.77489497744594108e-8)
    zz = z * z
    ps = ((f32(-1.9515295891e-4) * zz + f32(8.3321608736e-3)) * zz - f32(1.6666654611e-1)) * zz * z + z
    pc = ((f32(2.443315711809948e-5) * zz - f32(1.388731625493765e-3)) * zz + f32(4.166664568298827e-2)) * zz * zz \
        - f32(0.5) * zz + ONE
    if j == 0:
        return ps, pc
    if j == 2:
        return pc, -ps
    if j == 4:
        return -ps, -pc
    return -pc, ps


# ------------------------------------------------------------------ RNG, SH/PT_1_InitPass.wgsl:810-826

def GetHashValue(seed: int) -> int:
    state = (seed * 747796405 + 2891336453) & U32
    word = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & U32
    return ((word >> 22) ^ word) & U32


class Seed:
    """A `var rSeed : u32` passed by pointer."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v & U32


def Random(p: Seed):
    h = GetHashValue(p.v)
    p.v = (p.v + 1) & U32
    return f32(h) / f32(4294967295.0)


def Luminance(x):
    return dot(x, (f32(0.2126), f32(0.7152), f32(0.0722)))


# ------------------------------------------------------------------ the scene buffers, parsed as the shaders do

class Scene:
    """The bindings: UniformBuffer (33 words), SceneBuffer, GeometryBuffer, AccelBuffer."""

    def __init__(self, uniform, scene, geometry, accel):
        self.U = np.asarray(uniform, dtype=np.uint32)
        self.S = np.asarray(scene, dtype=np.uint32)
        self.Sf = self.S.view(np.float32)
        self.G = np.asarray(geometry, dtype=np.uint32)
        self.Gf = self.G.view(np.float32)
        self.A = np.asarray(accel, dtype=np.uint32)
        self.Af = self.A.view(np.float32)
        self.W, self.H = int(self.U[0]), int(self.U[1])
        self.frame_index = int(self.U[23])
        self.vpinv = [[f32(self.U[4:20].view(np.float32)[4 * c + r]) for r in range(4)] for c in range(4)]
        self._inst = {}
        self._desc = {}

    # GetInstance, SH/PT_1_InitPass.wgsl:244-268 (columns of the two matrices, MeshID)
    def instance(self, i):
        if i not in self._inst:
            o = STRIDE_INSTANCE * i
            m = [[self.Sf[o + 4 * c + r] for r in range(4)] for c in range(4)]
            mi = [[self.Sf[o + 16 + 4 * c + r] for r in range(4)] for c in range(4)]
            self._inst[i] = (m, mi, int(self.S[o + 32]))
        return self._inst[i]

    # GetMeshDescriptor, :270-283
    def descriptor(self, mesh):
        if mesh not in self._desc:
            o = int(self.U[24]) + STRIDE_DESCRIPTOR * mesh
            self._desc[mesh] = tuple(int(v) for v in self.S[o:o + 6])
        return self._desc[mesh]

    # GetMaterial, :285-314 (the transmissive albedo override and the roughness floor)
    def material(self, desc, mat_id):
        o = int(self.U[25]) + desc[2] + STRIDE_MATERIAL * mat_id
        w = self.Sf
        albedo = (w[o], w[o + 1], w[o + 2], w[o + 3])
        m = {"albedo": albedo, "metal": w[o + 8], "rough": w[o + 9], "trans": w[o + 10], "ior": w[o + 11]}
        if m["trans"] > Z:
            m["albedo"] = (ONE, ONE, Z, albedo[3])
        m["rough"] = fmax(m["rough"], f32(0.01))
        return m

    # GetLight, :324-340
    def light(self, lid):
        o = int(self.U[26]) + STRIDE_LIGHT * lid
        w = self.Sf
        return {"pos": (w[o], w[o + 1], w[o + 2]), "dir": (w[o + 3], w[o + 4], w[o + 5]),
                "color": (w[o + 6], w[o + 7], w[o + 8]), "U": (w[o + 9], w[o + 10], w[o + 11]),
                "V": (w[o + 12], w[o + 13], w[o + 14]), "type": int(self.S[o + 15]), "intensity": w[o + 16],
                "area": w[o + 17]}

    def cdf(self, idx):  # GetLightsCDF, :342-346
        return self.Sf[int(self.U[27]) + (idx & U32)]

    # GetBlasNode, :348-360: (min, max, offset, count)
    def blas(self, desc, sub, bid):
        root = int(self.G[int(self.U[29]) + desc[3] + sub])
        o = int(self.U[30]) + desc[4] + root + STRIDE_BLAS * bid
        a = self.Af
        return (a[o], a[o + 1], a[o + 2]), (a[o + 3], a[o + 4], a[o + 5]), int(self.A[o + 6]), int(self.A[o + 7])

    # GetVertex / GetTriangle, :362-388: three (position, normal) pairs
    def triangle(self, desc, prim):
        o = int(self.U[28]) + desc[1] + 3 * prim
        out = []
        for k in range(3):
            v = desc[0] + STRIDE_VERTEX * int(self.G[o + k])
            g = self.Gf
            out.append(((g[v], g[v + 1], g[v + 2]), (g[v + 3], g[v + 4], g[v + 5])))
        return out


def mat_vec(m, v4):
    """mat4x4 (columns) * vec4: sum over columns, left to right, no FMA."""
    return tuple(((m[0][r] * v4[0] + m[1][r] * v4[1]) + m[2][r] * v4[2]) + m[3][r] * v4[3] for r in range(4))


def matT_vec(m, v4):
    """transpose(m) * vec4: row r of the product is column r of m dotted with v."""
    return tuple(((m[r][0] * v4[0] + m[r][1] * v4[1]) + m[r][2] * v4[2]) + m[r][3] * v4[3] for r in range(4))


def TransformVec3WithMat4x4(v, m, transpose=False):  # :480-484
    t = (matT_vec if transpose else mat_vec)(m, (v[0], v[1], v[2], ONE))
    return (t[0] / t[3], t[1] / t[3], t[2] / t[3])


def TransformRayWithMat4x4(start, direction, m, bnormalize):  # :486-496
    s = TransformVec3WithMat4x4(start, m)
    e = TransformVec3WithMat4x4(vadd(start, direction), m)
    d = vsub(e, s)
    return s, (normalize(d) if bnormalize else d)


def GetRayAABBIntersectionRange(start, direction, bmin, bmax):  # :498-514
    inv = (ONE / direction[0], ONE / direction[1], ONE / direction[2])
    t1 = vmul(vsub(bmin, start), inv)
    t2 = vmul(vsub(bmax, start), inv)
    tmin_v = (fmin(t1[0], t2[0]), fmin(t1[1], t2[1]), fmin(t1[2], t2[2]))
    tmax_v = (fmax(t1[0], t2[0]), fmax(t1[1], t2[1]), fmax(t1[2], t2[2]))
    t_min = fmax(tmin_v[0], fmax(tmin_v[1], tmin_v[2]))
    t_max = fmin(tmax_v[0], fmin(tmax_v[1], tmax_v[2]))
    if t_min > t_max:
        return ONE, Z
    return t_min, t_max


def DoRangesOverlap(r1, r2):  # :475-478
    return (r1[0] <= r2[1]) and (r2[0] <= r1[1])


def GetRayTriangleHitDistance(start, direction, tri, det_eps):  # :516-547 (PT_01: 1e-8, :409)
    p0, p1, p2 = tri[0][0], tri[1][0], tri[2][0]
    e1 = vsub(p1, p0)
    e2 = vsub(p2, p0)
    pvec = cross(direction, e2)
    det = dot(e1, pvec)
    if abs(det) < det_eps:
        return INF
    inv_det = ONE / det
    tvec = vsub(start, p0)
    u = dot(tvec, pvec) * inv_det
    if u < Z or u > ONE:
        return INF
    qvec = cross(tvec, e1)
    v = dot(direction, qvec) * inv_det
    if v < Z or (u + v) > ONE:
        return INF
    t = dot(e2, qvec) * inv_det
    if t <= EPS:
        return INF
    return t


def GetBaryCentricWeights(p, A, B, C, eps):  # :549-575 (PT_01: 1e-6, :468)
    v0, v1, v2 = vsub(B, A), vsub(C, A), vsub(p, A)
    d00, d01, d11 = dot(v0, v0), dot(v0, v1), dot(v1, v1)
    d20, d21 = dot(v2, v0), dot(v2, v1)
    denom = d00 * d11 - d01 * d01
    if abs(denom) < eps:
        return ONE, Z, Z
    inv = ONE / denom
    u = (d11 * d20 - d01 * d21) * inv
    v = (d00 * d21 - d01 * d20) * inv
    w = ONE - u - v
    return w, u, v


class Pass:
    """The per-pass constants of TraceRay: PT_01 uses det 1e-8 / bary 1e-6, the others 1e-4 / 1e-8."""

    def __init__(self, det_eps, bary_eps):
        self.det_eps, self.bary_eps = f32(det_eps), f32(bary_eps)


GBUFFER_PASS = Pass(1e-8, 1e-6)
SHADING_PASS = Pass(1e-4, 1e-8)


def TraceRay(sc: Scene, ps: Pass, start, direction):
    """SH/PT_1_InitPass.wgsl:605-715 (PT_01:509-621): (valid, t, (inst, mat, prim, bary.x, bary.y))."""
    valid_range = [f32(1e-4), f32(1e10)]
    best = None
    for inst in range(int(sc.U[31])):
        m, mi, mesh = sc.instance(inst)
        desc = sc.descriptor(mesh)
        ls, ld = TransformRayWithMat4x4(start, direction, mi, False)
        for sub in range(desc[5]):
            bmin, bmax, _, _ = sc.blas(desc, sub, 0)
            if not DoRangesOverlap(valid_range, GetRayAABBIntersectionRange(ls, ld, bmin, bmax)):
                continue
            stack = [0]
            while stack:
                bid = stack.pop()
                bmin, bmax, off, cnt = sc.blas(desc, sub, bid)
                if not (cnt & 0xFFFF0000):
                    lc, rc = bid + 1, off // 8
                    lmin, lmax, _, _ = sc.blas(desc, sub, lc)
                    rmin, rmax, _, _ = sc.blas(desc, sub, rc)
                    lr = GetRayAABBIntersectionRange(ls, ld, lmin, lmax)
                    rr = GetRayAABBIntersectionRange(ls, ld, rmin, rmax)
                    hl, hr = DoRangesOverlap(valid_range, lr), DoRangesOverlap(valid_range, rr)
                    if hl and hr:
                        if lr[0] < rr[0]:
                            stack += [rc, lc]
                        else:
                            stack += [lc, rc]
                    elif hl:
                        stack.append(lc)
                    elif hr:
                        stack.append(rc)
                    continue
                for prim in range(off, off + (cnt & 0xFFFF)):
                    d = GetRayTriangleHitDistance(ls, ld, sc.triangle(desc, prim), ps.det_eps)
                    if valid_range[1] < d:
                        continue
                    valid_range[1] = d
                    best = (inst, sub, prim)
    if best is None:
        return False, Z, (0, 0, 0, Z, Z)
    t = valid_range[1]
    inst, sub, prim = best
    m, mi, mesh = sc.instance(inst)
    tri = sc.triangle(sc.descriptor(mesh), prim)
    A, B, C = (TransformVec3WithMat4x4(v[0], m) for v in tri)
    hit = vadd(start, sscale(t, direction))
    bw = GetBaryCentricWeights(hit, A, B, C, ps.bary_eps)
    return True, t, (inst, sub, prim, bw[0], bw[1])


def GetSurface(sc: Scene, cs):
    """SH/PT_1_InitPass.wgsl:438-467: (position, normal, material) of a CompactSurface."""
    inst, mat_id, prim, bx, by = cs
    m, mi, mesh = sc.instance(inst)
    desc = sc.descriptor(mesh)
    material = sc.material(desc, mat_id)
    tri = sc.triangle(desc, prim)
    P = [TransformVec3WithMat4x4(v[0], m) for v in tri]
    N = [TransformVec3WithMat4x4(v[1], mi, transpose=True) for v in tri]
    U, V = bx, by
    W = ONE - U - V
    n = normalize(vadd(vadd(vscale(N[0], U), vscale(N[1], V)), vscale(N[2], W)))
    p = vadd(vadd(vscale(P[0], U), vscale(P[1], V)), vscale(P[2], W))
    return {"pos": p, "n": n, "mat": material}


# ------------------------------------------------------------------ PBR, SH/PT_1_InitPass.wgsl:834-929

def GGXDistribution(ndoth, rough):
    alpha = rough * rough
    a2 = alpha * alpha
    x = ndoth * ndoth * (a2 - ONE) + ONE
    denom = PI * x * x
    return a2 / fmax(denom, EPS)


def GeometryShadow_Optimized(ndotv, ndotl, rough):
    r = rough + ONE
    k = r * r / f32(8.0)
    return ONE / ((ndotv * (ONE - k) + k) * (ndotl * (ONE - k) + k))


def Frensel(d, F0):
    p = pow5(ONE - saturate(d))
    return (F0[0] + (ONE - F0[0]) * p, F0[1] + (ONE - F0[1]) * p, F0[2] + (ONE - F0[2]) * p)


def BRDF(X, V, L):
    N = X["n"]
    H = normalize(vadd(L, V))
    ndotv, ndotl = fmax(dot(N, V), Z), fmax(dot(N, L), Z)
    ndoth, vdoth = fmax(dot(N, H), Z), fmax(dot(V, H), Z)
    base = X["mat"]["albedo"][:3]
    metal, rough = X["mat"]["metal"], X["mat"]["rough"]
    F0 = vmix((f32(0.04),) * 3, base, metal)
    D = GGXDistribution(ndoth, rough)
    G0 = GeometryShadow_Optimized(ndotv, ndotl, rough)
    F = Frensel(vdoth, F0)
    kD = vscale((ONE - F[0], ONE - F[1], ONE - F[2]), ONE - metal)
    diffuse = vmul(vdivs(kD, PI), base)
    spec = vscale(vscale(vscale(F, D), G0), f32(0.25))
    return vadd(diffuse, spec)


def BTDF(X, V, L):
    albedo = X["mat"]["albedo"][:3]
    rough, ior = X["mat"]["rough"], X["mat"]["ior"]
    same = dot(V, X["n"]) > Z
    n_in = ior if same else ONE
    n_out = ONE if same else ior
    h_norm = length(vadd(sscale(n_in, L), sscale(n_out, V)))
    N = X["n"] if same else vneg(X["n"])
    H = normalize(vadd(sscale(n_in, L), sscale(n_out, V)))
    ndotl, ndotv = abs(dot(N, L)), abs(dot(N, V))
    ndoth, ldoth, vdoth = abs(dot(N, H)), abs(dot(L, H)), abs(dot(V, H))
    G0 = GeometryShadow_Optimized(ndotl, ndotv, rough)
    D = GGXDistribution(ndoth, rough)
    nr = (n_out - n_in) / (n_out + n_in)
    F = Frensel(ldoth, (nr * nr,) * 3)
    # n_out * n_out * (1 - F) * LdotH * VdotH * G0 * D * Albedo, left to right
    s = n_out * n_out
    num = sscale(s, (ONE - F[0], ONE - F[1], ONE - F[2]))
    num = vscale(vscale(vscale(vscale(num, ldoth), vdoth), G0), D)
    num = vmul(num, albedo)
    return vdivs(num, fmax(h_norm * h_norm, EPS))


def BSDF(X, V, L):
    T = X["mat"]["trans"]
    N = X["n"]
    if dot(L, N) * dot(V, N) > Z:
        return sscale(ONE - T, BRDF(X, V, L))
    return sscale(T, BTDF(X, V, L))


# ------------------------------------------------------------------ sampling, :937-1106

def TBNMatrix(N):
    up, right = (Z, ONE, Z), (ONE, Z, Z)
    cv = right if abs(dot(N, up)) > f32(0.9999) else up
    T = normalize(cross(cv, N))
    B = cross(N, T)
    return T, B, N


def mat3_vec(tbn, v):  # mat3x3(T, B, N) * v = T v.x + B v.y + N v.z
    return vadd(vadd(vscale(tbn[0], v[0]), vscale(tbn[1], v[1])), vscale(tbn[2], v[2]))


def SampleCosineHemisphere(p: Seed):
    r1, r2 = Random(p), Random(p)
    R = np.sqrt(r1)
    phi = f32(2.0) * PI * r2
    s, c = sincos(phi)
    return R * c, R * s, np.sqrt(ONE - r1)


def SampleGGX(p: Seed, rough):
    r1, r2 = Random(p), Random(p)
    alpha = rough * rough
    phi = f32(2.0) * PI * r1
    cos_t = np.sqrt((ONE - r2) / (ONE + (alpha * alpha - ONE) * r2))
    sin_t = np.sqrt(ONE - cos_t * cos_t)
    s, c = sincos(phi)
    return normalize((sin_t * c, sin_t * s, cos_t))


def SampleNEE(sc: Scene, p: Seed, X, V, final_pass=False):
    P = Random(p)
    lo, hi = 0, int(sc.U[32]) - 1
    mid = (lo + hi) >> 1
    while lo < hi:
        if P < sc.cdf(mid):
            hi = mid
        else:
            lo = mid + 1
        mid = (lo + hi) >> 1
    L = sc.light(mid)
    xl = {"id": mid, "type": L["type"], "emit": sscale(L["intensity"], L["color"]), "pos": (Z, Z, Z),
          "dir": (Z, Z, Z), "pdf": Z}
    if L["type"] == LIGHT_DIRECTION:
        xl["pos"] = vsub(X["pos"], vscale(L["dir"], INF))
        xl["dir"] = L["dir"]
    elif L["type"] == LIGHT_POINT:
        xl["pos"] = L["pos"]
        xl["dir"] = normalize(vsub(X["pos"], L["pos"]))
    elif L["type"] == LIGHT_RECT:
        ru = Random(p) * f32(2.0) - ONE
        rv = Random(p) * f32(2.0) - ONE
        off = vadd(sscale(ru, L["U"]), sscale(rv, L["V"]))
        xl["pos"] = vadd(L["pos"], off)
        xl["dir"] = normalize(vsub(X["pos"], xl["pos"]))
    xl["pdf"] = PDF_LIGHT(sc, X, V, xl, final_pass)
    return xl


def SampleBRDF(p: Seed, X, V):
    albedo, metal, rough = X["mat"]["albedo"][:3], X["mat"]["metal"], X["mat"]["rough"]
    F0 = vmix((f32(0.04),) * 3, albedo, metal)
    p_spec = mix(Luminance(F0), ONE, metal)
    tbn = TBNMatrix(X["n"])
    spec = Random(p) < p_spec
    if spec:
        H = mat3_vec(tbn, SampleGGX(p, rough))
        L = reflect(vneg(V), H)
    else:
        L = mat3_vec(tbn, SampleCosineHemisphere(p))
    return L, (LOBE_GGX if spec else LOBE_LAMBERT)


def SampleBTDF(p: Seed, X, V):
    STATS["btdf_sample"] += 1
    same = dot(V, X["n"]) > Z
    ior = X["mat"]["ior"]
    n_in = ONE if same else ior
    n_out = ior if same else ONE
    N = X["n"] if same else vneg(X["n"])
    ratio = n_in / n_out
    r = (ONE - ratio) / (ONE + ratio)
    R2 = ratio * ratio
    cos_t = abs(dot(V, N))
    p_refl = Frensel(cos_t, (r * r,) * 3)[0]
    if cos_t * cos_t < (R2 - ONE) / R2:
        p_refl = ONE
    refl = Random(p) < p_refl
    tbn = TBNMatrix(N)
    H = mat3_vec(tbn, SampleGGX(p, X["mat"]["rough"]))
    L = normalize(reflect(vneg(V), H) if refl else refract(vneg(V), H, ratio))
    return L, LOBE_GGX


def SampleBSDF(p: Seed, X, V):
    if Random(p) < X["mat"]["trans"]:
        return SampleBTDF(p, X, V)
    return SampleBRDF(p, X, V)


# ------------------------------------------------------------------ PDFs, :1114-1245

def PDF_BRDF(X, V, L):
    albedo, metal, rough = X["mat"]["albedo"][:3], X["mat"]["metal"], X["mat"]["rough"]
    F0 = vmix((f32(0.04),) * 3, albedo, metal)
    p_spec = mix(Luminance(F0), ONE, metal)
    N = X["n"]
    H = normalize(vadd(L, V))
    ldotn, ndoth, vdoth = fmax(dot(L, N), Z), fmax(dot(N, H), Z), fmax(dot(V, H), Z)
    pdf_spec = GGXDistribution(ndoth, rough) / fmax(f32(4.0) * vdoth, EPS)
    pdf_diff = ldotn / PI
    return mix(pdf_diff, pdf_spec, p_spec)


def PDF_BTDF(X, V, L):
    rough, ior = X["mat"]["rough"], X["mat"]["ior"]
    same = dot(V, X["n"]) > Z
    n_in = ONE if same else ior
    n_out = ior if same else ONE
    ratio = n_in / n_out
    N = X["n"] if same else vneg(X["n"])
    r0 = (ONE - ratio) / (ONE + ratio)
    R0 = r0 * r0
    cos_t = abs(dot(V, N))
    p_refl = Frensel(cos_t, (R0,) * 3)[0]
    sin2 = ONE - cos_t * cos_t
    if sin2 * (ratio * ratio) > ONE:
        p_refl = ONE
    p_trans = ONE - p_refl
    pdf_r = Z
    if p_refl > Z:
        Hr = normalize(vadd(V, L))
        ndoth, vdoth = fmax(Z, dot(N, Hr)), fmax(Z, dot(V, Hr))
        if vdoth > Z:
            pdf_r = GGXDistribution(ndoth, rough) / (f32(4.0) * vdoth)
    pdf_t = Z
    if p_trans > Z:
        Ht = normalize(vadd(vscale(V, n_out), vscale(L, n_in)))
        ndoth, vdoth, ldoth = fmax(Z, dot(N, Ht)), fmax(Z, dot(V, Ht)), fmax(Z, dot(L, Ht))
        denom = n_in * ldoth + n_out * vdoth
        if denom > Z:
            J = (n_out * n_out * vdoth) / (denom * denom)
            pdf_t = GGXDistribution(ndoth, rough) * abs(J)
    return p_refl * pdf_r + p_trans * pdf_t


def PDF_BSDF(X, V, L):
    N = X["n"]
    if dot(L, N) * dot(V, N) > Z:
        return PDF_BRDF(X, V, L)
    return PDF_BTDF(X, V, L)


def DirectionToLight(X, xl):  # :746-772
    t = xl["type"]
    if t in (LIGHT_DIRECTION, LIGHT_ENV):
        return vneg(xl["dir"])
    if t in (LIGHT_POINT, LIGHT_RECT):
        return normalize(vsub(xl["pos"], X["pos"]))
    return (Z, Z, Z)


def PDF_LIGHT(sc: Scene, X, V, xl, final_pass=False):
    """:1220-1245; PT_4 (final_pass) divides by A |N.L| without the EPS floor
    (SH/PT_4_FinalShadingPass.wgsl:1249)."""
    if xl["type"] == LIGHT_ENV:
        return PDF_BSDF(X, V, DirectionToLight(X, xl))
    lid = xl["id"]
    L = sc.light(lid)
    before = Z if lid == 0 else sc.cdf(lid - 1)
    choose = sc.cdf(lid) - before
    pdf_point = ONE
    if xl["type"] == LIGHT_RECT:
        r = vsub(xl["pos"], X["pos"])
        Ld = normalize(r)
        den = L["area"] * abs(dot(L["dir"], Ld))
        pdf_point = dot(r, r) / (den if final_pass else fmax(den, EPS))
    return choose * pdf_point


def L_emit(xl, X, final_pass=False):  # :1253-1260 (PT_4: no EPS floor, :1265)
    r = vsub(xl["pos"], X["pos"])
    rr = dot(r, r)
    att = (ONE / (rr if final_pass else fmax(rr, EPS))) if xl["type"] == LIGHT_POINT else ONE
    return vscale(xl["emit"], att)


def Visibility(sc: Scene, start, end):  # :774-802 (the full closest-hit range, every segment)
    T = ONE
    dist = length(vsub(end, start))
    direction = vdivs(vsub(end, start), dist)
    cur = start
    remain = dist
    for _ in range(5):
        ok, t, cs = TraceRay(sc, SHADING_PASS, cur, direction)
        if not ok or t > remain:
            return T
        m, mi, mesh = sc.instance(cs[0])
        trans = sc.material(sc.descriptor(mesh), cs[1])["trans"]
        if trans == Z:
            return Z
        T = T * trans
        remain = remain - t
        cur = GetSurface(sc, cs)["pos"]
        STATS["visibility_through_transmissive"] += 1
    return Z


def CreateEnvLight(X, V, L):  # :717-730
    STATS["env_path"] += 1
    return {"id": -1, "type": LIGHT_ENV, "emit": ENV, "pos": vadd(X["pos"], vscale(L, INF)), "dir": vneg(L),
            "pdf": PDF_BSDF(X, V, L)}


def IsSafeToReconnect(A, la, B, lb):  # :1262-1271
    ra = ONE if la == LOBE_LAMBERT else A["mat"]["rough"]
    rb = ONE if lb == LOBE_LAMBERT else B["mat"]["rough"]
    rough = fmin(ra, rb) >= f32(0.5)
    far = length(vsub(A["pos"], B["pos"])) >= f32(0.1)
    return far and rough


def IsSafeToReconnect_Light(X, xl):  # :1273-1281
    rough = X["mat"]["rough"] >= f32(0.5)
    directional = xl["type"] in (LIGHT_DIRECTION, LIGHT_ENV)
    far = directional or (length(vsub(X["pos"], xl["pos"])) >= f32(0.1))
    return far and rough


ZERO_SURFACE = {"pos": (Z, Z, Z), "n": (Z, Z, Z),
                "mat": {"albedo": (Z, Z, Z, Z), "metal": Z, "rough": Z, "trans": Z, "ior": Z}}
ZERO_XL = {"id": 0, "type": 0, "emit": (Z, Z, Z), "pos": (Z, Z, Z), "dir": (Z, Z, Z), "pdf": Z}


def new_path():
    """Path() -- WGSL zero-initialises function-scope variables."""
    return {"surf": [ZERO_SURFACE] * 8, "lobe": [0] * 8, "seed": [0] * 8, "xl": ZERO_XL, "length": 0}


def copy_path(p):
    return {"surf": list(p["surf"]), "lobe": list(p["lobe"]), "seed": list(p["seed"]), "xl": p["xl"],
            "length": p["length"]}


def SafeReconnectionIndex(path):  # :1283-1296 (array reads clamped to [0, 7])
    n = path["length"]
    for k in range(2, n):
        if IsSafeToReconnect(path["surf"][k - 1], path["lobe"][k - 1], path["surf"][k], path["lobe"][k]):
            return k
    last = min((n - 1) & U32, 7)
    if IsSafeToReconnect_Light(path["surf"][last], path["xl"]):
        return n
    return 0


def xl_words(xl):
    """LightSample in the CompactPath layout: Direction, Type, Position, LightID, Emittance, PDF."""
    f = np.array([*xl["dir"], Z, *xl["pos"], Z, *xl["emit"], xl["pdf"]], dtype=np.float32).view(np.uint32)
    f[3] = xl["type"] & U32
    f[7] = xl["id"] & U32
    return f


def rc_vertex(cs):  # GetRcVertex, :409-422
    inst, mat, prim, bx, by = cs
    w = np.array([0, 0, bx, by], dtype=np.float32).view(np.uint32)
    w[0] = (1 << 31) | (inst << 16) | mat
    w[1] = prim
    return w


def CompressPath(path, csurf):  # :1322-1353 -> the 28 CompactPath words
    w = np.zeros(28, dtype=np.uint32)
    k = SafeReconnectionIndex(path)
    w[0:4] = [s & U32 for s in path["seed"][2:6]]
    w[4:16] = xl_words(path["xl"])
    w[20] = k
    w[23] = path["length"]
    if k == 0:
        STATS["unshiftable_path"] += 1
        return w
    STATS["reconnection_light" if k == path["length"] else "reconnection_vertex"] += 1
    is_light = k == path["length"]
    w[22] = LOBE_LIGHT if is_light else path["lobe"][k]
    w[21] = path["lobe"][k - 1]
    if not is_light:
        w[16:20] = rc_vertex(csurf[k])
    return w


def Get_X0(sc: Scene, x, y):  # :732-738
    u = (f32(x) + f32(0.5)) / f32(sc.W)
    v = (f32(y) + f32(0.5)) / f32(sc.H)
    ndc = (f32(2.0) * u - ONE, f32(2.0) * v - ONE, Z)
    return TransformVec3WithMat4x4(ndc, sc.vpinv)


def gbuffer_pixel(sc: Scene, x, y):
    """PT_01 cs_main (SH/PT_01_GBufferPass.wgsl:628-659, GenerateRayFromThreadID :496-507):
    the G-buffer texel as 4 u32 words, and the CompactSurface Get_X1 decodes from it."""
    with np.errstate(all="ignore"):
        return _gbuffer_pixel(sc, x, y)


def _gbuffer_pixel(sc: Scene, x, y):
    u = (f32(x) + f32(0.5)) / f32(sc.W)
    v = (f32(y) + f32(0.5)) / f32(sc.H)
    ndc = (f32(2.0) * u - ONE, f32(2.0) * v - ONE, Z)
    s, d = TransformRayWithMat4x4(ndc, (Z, Z, ONE), sc.vpinv, True)
    ok, t, cs = TraceRay(sc, GBUFFER_PASS, s, d)
    inst, mat, prim, bx, by = cs
    w = np.array([0, 0, bx, by], dtype=np.float32).view(np.uint32)
    w[0] = ((1 if ok else 0) << 31) | (inst << 16) | mat
    w[1] = prim
    return w, ok, cs


def UpdateReservoir(p: Seed, R, sample, ris, p_hat, conf):  # :1298-1320
    R["C"] += conf
    R["w_sum"] = R["w_sum"] + ris
    pr = ris / R["w_sum"]
    if not (Random(p) < pr):
        return
    R["sample"] = copy_path(sample)
    R["p_hat"] = p_hat


def init_pixel(sc: Scene, x, y, gb_cs):
    """PT_1 cs_main (SH/PT_1_InitPass.wgsl:1361-1486): the 32 reservoir words of pixel (x, y)."""
    seed = Seed(GetHashValue((x * 1973 + y * 9277 + sc.frame_index * 26699) & U32))
    f = (ONE, ONE, ONE)
    p = ONE
    csurf = [(0, 0, 0, Z, Z)] * 8
    csurf[1] = gb_cs
    R = {"w_sum": Z, "C": 0, "sample": new_path(), "p_hat": Z}
    path = new_path()
    path["surf"][0] = dict(ZERO_SURFACE, pos=Get_X0(sc, x, y))
    path["surf"][1] = GetSurface(sc, gb_cs)
    path["length"] = 2
    with np.errstate(all="ignore"):
        for i in (1, 2, 3):
            X = path["surf"][i]
            V = normalize(vsub(path["surf"][i - 1]["pos"], X["pos"]))
            # NEE
            path["seed"][i + 1] = seed.v
            path["xl"] = SampleNEE(sc, seed, X, V)
            L = DirectionToLight(X, path["xl"])
            c = vmul(f, L_emit(path["xl"], X))
            c = vmul(c, BSDF(X, V, L))
            c = vscale(c, abs(dot(X["n"], L)))
            c = vscale(c, Visibility(sc, X["pos"], path["xl"]["pos"]))
            p_hat = Luminance(c)
            ris = p_hat / (p * path["xl"]["pdf"])
            UpdateReservoir(seed, R, path, ris, p_hat, 1)
            if i == 3:
                break
            # BSDF sample
            path["seed"][i + 1] = seed.v
            L, lobe = SampleBSDF(seed, X, V)
            path["lobe"][i] = lobe
            f = vmul(f, vscale(BSDF(X, V, L), abs(dot(X["n"], L))))  # f *= BSDF(..) * abs(..)
            p = p * PDF_BSDF(X, V, L)
            p_surv = Luminance(f) / p
            if Random(seed) < p_surv:
                p = p * p_surv
            else:
                STATS["russian_roulette_end"] += 1
                break
            ok, t, cs = TraceRay(sc, SHADING_PASS, X["pos"], L)
            if not ok:
                path["xl"] = CreateEnvLight(X, V, L)
                c = vmul(f, ENV)
                p_hat = Luminance(c)
                UpdateReservoir(seed, R, path, p_hat / p, p_hat, 1)
                break
            csurf[i + 1] = cs
            path["surf"][i + 1] = GetSurface(sc, cs)
            path["length"] += 1
        out = np.zeros(32, dtype=np.uint32)
        out[0:28] = CompressPath(R["sample"], csurf)
        out[28] = np.array([R["w_sum"] / R["p_hat"]], dtype=np.float32).view(np.uint32)[0]
        out[29] = R["C"]
    return out


def decode_xl(w):
    f = w.view(np.float32)
    return {"dir": (f[4], f[5], f[6]), "type": int(w[7]), "pos": (f[8], f[9], f[10]),
            "id": int(np.int32(w[11])), "emit": (f[12], f[13], f[14]), "pdf": f[15]}


def final_pixel(sc: Scene, x, y, gb_words, gb_cs, res_words, scene_color):
    """PT_4 cs_main (SH/PT_4_FinalShadingPass.wgsl:1392-1428) + WriteColor (:599-605): the
    pixel's new Scene texel (rgba f32) from the accumulated one."""
    with np.errstate(all="ignore"):
        if not (int(gb_words[0]) & 0x80000000):
            return np.array([*ENV, ONE], dtype=np.float32)

        def write(c):
            t = ONE / f32(sc.frame_index + 1)
            return np.array([mix(f32(scene_color[k]), c[k], t) for k in range(3)] + [ONE], dtype=np.float32)
        C, length_ = int(res_words[29]), int(res_words[23])
        if C == 0 or length_ < 2:
            return write((Z, Z, Z))
        ucw = res_words[28:29].view(np.float32)[0]
        xl = decode_xl(res_words)
        seeds = [int(s) for s in res_words[0:4]]
        # RegeneratePath (:1357-1384)
        surf = [None] * 8
        surf[0] = dict(ZERO_SURFACE, pos=Get_X0(sc, x, y))
        surf[1] = GetSurface(sc, gb_cs)
        STATS[f"pt4_replay_length_{length_}"] += 1
        for i in range(1, length_ - 1):
            V = normalize(vsub(surf[i - 1]["pos"], surf[i]["pos"]))
            s = Seed(seeds[min(i - 1, 3)])
            L, _ = SampleBSDF(s, surf[i], V)
            ok, t, cs = TraceRay(sc, SHADING_PASS, surf[i]["pos"], L)
            surf[i + 1] = GetSurface(sc, cs)  # (a miss decodes instance 0's triangle 0, as the WGSL does)
        # PathContribution (:1306-1336): BSDF(X, L, V) -- V and L swapped in the calls, as written
        f = (ONE, ONE, ONE)
        for i in range(1, length_ - 1):
            V = normalize(vsub(surf[i - 1]["pos"], surf[i]["pos"]))
            L = normalize(vsub(surf[i + 1]["pos"], surf[i]["pos"]))
            f = vmul(f, vscale(BSDF(surf[i], L, V), abs(dot(surf[i]["n"], L))))
        Xp, Xc = surf[length_ - 2], surf[length_ - 1]
        V = normalize(vsub(Xp["pos"], Xc["pos"]))
        L = DirectionToLight(Xc, xl)
        f = vmul(f, vscale(BSDF(Xc, L, V), abs(dot(Xc["n"], L))))
        f = vmul(f, vscale(L_emit(xl, Xc, final_pass=True), Visibility(sc, Xc["pos"], xl["pos"])))
        return write(sscale(ucw, f))


def mcpt_pixel(sc: Scene, x, y, scene_color):
    """TEST_MCPT cs_main (SH/TEST_MCPT.wgsl:1315-1372, GetLightColor :1261-1309, WriteColor
    :596-602): the brute-force path tracer's new Scene texel of pixel (x, y)."""
    with np.errstate(all="ignore"):
        seed = Seed(GetHashValue((x * 1973 + y * 9277 + sc.frame_index * 26699) & U32))
        u = (f32(x) + f32(0.5)) / f32(sc.W)
        v = (f32(y) + f32(0.5)) / f32(sc.H)
        ndc = (f32(2.0) * u - ONE, f32(2.0) * v - ONE, Z)
        start, direction = TransformRayWithMat4x4(ndc, (Z, Z, ONE), sc.vpinv, True)
        color = (Z, Z, Z)
        f = (ONE, ONE, ONE)
        p = ONE
        for _ in range(3):
            ok, t, cs = TraceRay(sc, SHADING_PASS, start, direction)
            if not ok:
                color = vadd(color, vmul(vdivs(f, p), ENV))
                break
            X = GetSurface(sc, cs)
            V = normalize(vsub(start, X["pos"]))
            for lid in range(int(sc.U[32])):
                color = vadd(color, vmul(vdivs(f, p), light_color(sc, seed, X, V, lid)))
            L, _ = SampleBSDF(seed, X, V)
            f = vmul(f, vscale(BSDF(X, V, L), abs(dot(X["n"], L))))
            p = p * PDF_BSDF(X, V, L)
            start, direction = X["pos"], L
            p_surv = Luminance(f) / p
            if Random(seed) < p_surv:
                p = p * p_surv
            else:
                break
        t = ONE / f32(sc.frame_index + 1)
        return np.array([mix(f32(scene_color[k]), color[k], t) for k in range(3)] + [ONE], dtype=np.float32)


def light_color(sc: Scene, seed: Seed, X, V, lid):
    """GetLightColor (SH/TEST_MCPT.wgsl:1261-1309): every light once, PDF 1 for delta lights."""
    L = sc.light(lid)
    xl = {"id": lid, "type": L["type"], "emit": sscale(L["intensity"], L["color"]), "pos": (Z, Z, Z),
          "dir": (Z, Z, Z), "pdf": Z}
    if L["type"] == LIGHT_DIRECTION:
        xl["pos"] = vsub(X["pos"], vscale(L["dir"], INF))
        xl["dir"] = L["dir"]
        xl["pdf"] = ONE
    elif L["type"] == LIGHT_POINT:
        xl["pos"] = L["pos"]
        xl["dir"] = normalize(vsub(X["pos"], L["pos"]))
        xl["pdf"] = ONE
    elif L["type"] == LIGHT_RECT:
        ru = Random(seed) * f32(2.0) - ONE
        rv = Random(seed) * f32(2.0) - ONE
        xl["pos"] = vadd(L["pos"], vadd(sscale(ru, L["U"]), sscale(rv, L["V"])))
        xl["dir"] = normalize(vsub(X["pos"], xl["pos"]))
        r = vsub(xl["pos"], X["pos"])
        Ld = normalize(r)
        xl["pdf"] = dot(r, r) / fmax(L["area"] * abs(dot(L["dir"], Ld)), EPS)
    Ld = DirectionToLight(X, xl)
    c = vmul(L_emit(xl, X), BSDF(X, V, Ld))
    c = vscale(c, abs(dot(X["n"], Ld)))
    c = vscale(c, Visibility(sc, X["pos"], xl["pos"]))
    return vdivs(c, xl["pdf"])
