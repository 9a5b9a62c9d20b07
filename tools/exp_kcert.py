"""Dev (CPU, numpy): how many of the sampler's 0.5 km scan steps a certificate that bounds the
k-parallel factor would certify, against the step certificate of sample_kernel (DESIGN.md §3
sample_kernel). Lines are drawn like find_samples_new's (RayTracer.jl:1486-1531; numpy's RNG,
not Philox: a statistical sample). The condition is evaluated in the closed form
    ½(ωp² (1 - κ c²) - m_a²)/E²,  ωp² = wp2n |ẑ·G| / |x|⁵,  c² = (v̂l·G)² / (|x|² (3 M² + |x|²)),
    G = 3 M x - |x|² m̂,  M = m̂·x,  κ = 1 - (1 - rs/r) m_a²/E²,
which equals sampler_condition_e outside r = 10 km (checked against the oracle below).
Usage: python tools/exp_kcert.py [lines] [maxR-config: flat|scan]"""
import sys

import numpy as np

C_KM, HBAR, GNEW, PI = 2.99792e5, 6.582119e-16, 132712000000.0, np.pi


def kparams(theta_m=0.2, omega_pul=1.0, B0=1e14, rNS=10.0, mass_ns=1.0, mass_a=1e-5):
    ne_coef = abs(2.0 * omega_pul / np.sqrt(4.0 * PI / 137.0) * 1.95e-2 * HBAR)
    wp2_coef = 4.0 * PI * ne_coef / 137.0 / 5.0e5
    return dict(cm=np.cos(theta_m), sm=np.sin(theta_m), wp2n=wp2_coef * abs(0.5 * B0 * rNS ** 3), rNS=rNS,
                rs=2.0 * GNEW * mass_ns / C_KM ** 2, ma=mass_a, ma2=mass_a * mass_a)


def cond(P, x, vl, E):
    """closed form of the condition (without the ½/E² factor), x (..., 3), vl (..., 3)"""
    mh = np.array([P["sm"], 0.0, P["cm"]])
    R2 = (x * x).sum(-1)
    M = x @ mh
    G = 3.0 * M[..., None] * x - R2[..., None] * mh
    r = np.sqrt(R2)
    wp2 = P["wp2n"] * np.abs(G[..., 2]) / (R2 * R2 * r)
    c2 = (vl * G).sum(-1) ** 2 / (R2 * (3.0 * M * M + R2))
    kap = 1.0 - (1.0 - P["rs"] / r) * P["ma2"] / (E * E)
    return wp2 * (1.0 - kap * c2) - P["ma2"]


def quad_range(c0, c1, c2, sa, sb):
    fa = c0 + sa * (c1 + sa * c2)
    fb = c0 + sb * (c1 + sb * c2)
    lo, hi = np.minimum(fa, fb), np.maximum(fa, fb)
    with np.errstate(divide="ignore", invalid="ignore"):
        sv = -c1 / (2.0 * c2)
    inside = (c2 != 0.0) & (sv > sa) & (sv < sb)
    fv = c0 + sv * (c1 + sv * c2)
    lo = np.where(inside, np.minimum(lo, fv), lo)
    hi = np.where(inside, np.maximum(hi, fv), hi)
    return lo, hi


def abs_range(lo, hi):
    alo = np.where(lo > 0, lo, np.where(hi < 0, -hi, 0.0))
    ahi = np.maximum(np.abs(lo), np.abs(hi))
    return alo, ahi


def basic_cert(P, X0, VA, E, sa, sb):
    """sample_kernel's seg_cert: 1 negative, 2 positive, 0 none"""
    sd = -(X0 * VA).sum(-1)
    sm_ = np.clip(sd, sa, sb)
    xm = X0 + VA * sm_[..., None]
    rm2 = (xm * xm).sum(-1)
    rmin = np.sqrt(rm2)
    xa, xb = X0 + VA * sa[..., None], X0 + VA * sb[..., None]
    ra2, rb2 = (xa * xa).sum(-1), (xb * xb).sum(-1)
    ba = (P["cm"] * (3 * xa[..., 2] ** 2 - ra2) + 3 * P["sm"] * xa[..., 0] * xa[..., 2]) / ra2
    bb = (P["cm"] * (3 * xb[..., 2] ** 2 - rb2) + 3 * P["sm"] * xb[..., 0] * xb[..., 2]) / rb2
    al = (sb - sa) / rmin
    db = 0.75 * al * al * (1 + 1e-9) + 1e-12
    bmax = np.minimum(2.0, np.maximum(np.abs(ba), np.abs(bb)) + db)
    neg = 2.0 * P["wp2n"] * 0.5 * bmax < P["ma2"] * (1 - 1e-6) * (rm2 * rmin)
    bmin = np.where(ba * bb > 0, np.minimum(np.abs(ba), np.abs(bb)) - db, -1.0)
    rmax2 = np.maximum(ra2, rb2)
    grr = 1.0 - P["rs"] / rmin * (1 + 1e-15)
    pos = (rmin > 10.0) & (bmin > 0) & (P["wp2n"] * bmin * grr > E * E * (1 + 1e-6) * rmax2 * np.sqrt(rmax2))
    return np.where(neg, 1, np.where(pos, 2, 0))


def k_cert(P, X0, VA, VL, E, sa, sb):
    """the k-parallel-aware certificate on [sa, sb]: exact ranges of the quadratics in s, then intervals"""
    mh = np.array([P["sm"], 0.0, P["cm"]])
    r0, r1, r2 = (X0 * X0).sum(-1), 2.0 * (X0 * VA).sum(-1), (VA * VA).sum(-1)
    m0, m1 = X0 @ mh, VA @ mh
    z0, z1 = X0[..., 2], VA[..., 2]
    l0, l1 = (VL * X0).sum(-1), (VL * VA).sum(-1)
    vm = VL @ mh
    Z = (3 * z0 * m0 - P["cm"] * r0, 3 * (z0 * m1 + z1 * m0) - P["cm"] * r1, 3 * z1 * m1 - P["cm"] * r2)
    V = (3 * l0 * m0 - vm * r0, 3 * (l0 * m1 + l1 * m0) - vm * r1, 3 * l1 * m1 - vm * r2)
    R2lo, R2hi = quad_range(r0, r1, r2, sa, sb)
    Zlo, Zhi = abs_range(*quad_range(*Z, sa, sb))
    Vlo, Vhi = abs_range(*quad_range(*V, sa, sb))
    Mlo, Mhi = abs_range(m0 + m1 * sa, m0 + m1 * sb) if True else None
    Mlo, Mhi = abs_range(np.minimum(m0 + m1 * sa, m0 + m1 * sb), np.maximum(m0 + m1 * sa, m0 + m1 * sb))
    rlo, rhi = np.sqrt(R2lo), np.sqrt(R2hi)
    wlo = P["wp2n"] * Zlo / (R2hi * R2hi * rhi)
    whi = P["wp2n"] * Zhi / (R2lo * R2lo * rlo)
    clo = Vlo * Vlo / (R2hi * (3 * Mhi * Mhi + R2hi))
    chi = np.minimum(1.0, Vhi * Vhi / (R2lo * (3 * Mlo * Mlo + R2lo)))
    iE2 = 1.0 / (E * E)
    klo = 1.0 - (1.0 - P["rs"] / rhi) * P["ma2"] * iE2
    khi = 1.0 - (1.0 - P["rs"] / rlo) * P["ma2"] * iE2
    neg = whi * (1 + 1e-9) * (1.0 - klo * clo) < P["ma2"] * (1 - 1e-6)
    pos = wlo * (1 - 1e-9) * (1.0 - khi * chi) > P["ma2"] * (1 + 1e-6)
    ok = rlo > max(10.0, P["rNS"])
    return np.where(ok & neg, 1, np.where(ok & pos, 2, 0))


def lines(P, n, maxR, rng):
    U = rng.random((n, 10))
    cti = 1 - 2 * U[:, 0]; sti = np.sqrt((1 - cti) * (1 + cti))
    phi = U[:, 1] * 2 * PI
    ctl = 1 - 2 * U[:, 2]; stl = np.sqrt((1 - ctl) * (1 + ctl))
    phl = U[:, 3] * 2 * PI
    pR = U[:, 4] * 2 * PI
    rR = np.sqrt(U[:, 5]) * maxR
    va = np.stack([sti * np.cos(phi), sti * np.sin(phi), cti], -1)
    vl = np.stack([stl * np.cos(phl), stl * np.sin(phl), ctl], -1)
    x1, x2 = rR * np.cos(pR), rR * np.sin(pR)
    cp, sp = np.cos(phi), np.sin(phi)
    x0 = np.stack([x1 * cp * cti - x2 * sp, x2 * cp + x1 * sp * cti, -x1 * sti], -1)
    vI = (220.0 + U[:, 6:9] * 1e-5) / np.sqrt(3.0)
    vmag = np.sqrt((vI * vI).sum(-1))
    g = 1 / np.sqrt(1 - (vmag / C_KM) ** 2)
    E = P["ma"] * np.sqrt(1 + (vmag / C_KM * g) ** 2)
    x0 = x0 + va * (-maxR * 1.1)
    return x0, va, vl, E


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    which = sys.argv[2] if len(sys.argv) > 2 else "flat"
    P = kparams() if which == "flat" else kparams(theta_m=0.0, mass_a=1e-5, B0=2e14, omega_pul=2 * PI)
    # maxR: the conversion radius at the pole direction, Find_Conversion_Surface's value for the flat config
    maxR = float(sys.argv[3]) if len(sys.argv) > 3 else 25.167098523268997
    rng = np.random.default_rng(1)
    X0, VA, VL, E = lines(P, n, maxR, rng)
    send = 2.2 * maxR
    nst = int(np.ceil(send / 0.5))
    jj = np.arange(1, 20) / 19.0
    tot = dict(steps=0, basic_unc=0, k_unc=0, sub2=0, sub4=0, bad=0, brackets=0)
    sub_pts = {2: 0, 4: 0}
    for st in range(nst):
        s0 = np.full(n, st * 0.5)
        s1 = np.minimum(s0 + 0.5, send)
        pts = s0[:, None] + (s1 - s0)[:, None] * jj[None, :]
        xs = X0[:, None, :] + VA[:, None, :] * pts[..., None]
        v = cond(P, xs, VL[:, None, :], E[:, None])
        bc = basic_cert(P, X0, VA, E, s0, s1)
        kc = k_cert(P, X0, VA, VL, E, s0, s1)
        c = np.where(bc > 0, bc, kc)
        # soundness on the evaluated points
        bad = ((c == 1) & (v >= 0).any(1)) | ((c == 2) & (v <= 0).any(1))
        tot["bad"] += int(bad.sum())
        tot["steps"] += n
        tot["basic_unc"] += int((bc == 0).sum())
        tot["k_unc"] += int((c == 0).sum())
        tot["brackets"] += int((np.diff(np.signbit(v).astype(int), axis=1) != 0).sum())
        for K in (2, 4):
            u = c == 0
            for q in range(K):
                a_j, b_j = (19 * q) // K, (19 * (q + 1)) // K  # points (a_j, b_j] of the step
                sa = s0 + (s1 - s0) * a_j / 19.0
                sb = s0 + (s1 - s0) * b_j / 19.0
                cq = np.where(basic_cert(P, X0, VA, E, sa, sb) > 0, 1, k_cert(P, X0, VA, VL, E, sa, sb))
                sub_pts[K] += int(((cq == 0) & u).sum()) * (b_j - a_j)
    print({**tot, "points_basic": tot["basic_unc"] * 19, "points_k": tot["k_unc"] * 19,
           "points_sub2": sub_pts[2], "points_sub4": sub_pts[4]})


if __name__ == "__main__":
    main()
