"""Derive the fp64 constants of mpc_trig.h with mpmath (run once; output is
pasted into diplomjourney_amd/csrc/mpc_trig.h).

* Cody-Waite split of pi/2: P1 (33 significant bits), P2 (next 33 bits),
  P3 (the next 53 bits), so that k*P1 and k*P2 are exact for |k| < 2^20.
* Near-minimax (Chebyshev) polynomials on the reduced interval |r| <= pi/4:
    sin(r) = r + r^3 * S(r^2)
    cos(r) = 1 - r^2/2 + r^4 * C(r^2)
    tan(r) = r + r^3 * T(r^2)
"""
import mpmath as mp

mp.mp.prec = 256


def split(x, bits):
    """Round x to `bits` significant bits (toward zero) and return (hi, rest)."""
    e = mp.floor(mp.log(abs(x), 2))
    scale = mp.mpf(2) ** (bits - 1 - e)
    hi = mp.floor(x * scale) / scale
    return hi, x - hi


def d(x):
    return float(x)


def main():
    pio2 = mp.pi / 2
    p1, rest = split(pio2, 33)
    p2, rest2 = split(rest, 33)
    p3 = rest2
    print("// Cody-Waite pi/2 = P1 + P2 + P3")
    for name, v in (("P1", p1), ("P2", p2), ("P3", p3)):
        print(f"constexpr double k{name} = {d(v).hex()};  // {mp.nstr(v, 25)}")
    print(f"constexpr double kTwoOverPi = {d(2 / mp.pi).hex()};")
    a = (mp.pi / 4) * (1 + mp.mpf("1e-6"))
    s_max = a * a

    def S(s):
        if s == 0:
            return -mp.mpf(1) / 6
        r = mp.sqrt(s)
        return (mp.sin(r) - r) / (r * s)

    def C(s):
        if s == 0:
            return mp.mpf(1) / 24
        r = mp.sqrt(s)
        return (mp.cos(r) - 1 + s / 2) / (s * s)

    def T(s):
        if s == 0:
            return mp.mpf(1) / 3
        r = mp.sqrt(s)
        return (mp.tan(r) - r) / (r * s)

    for name, fn, deg in (("S", S, 6), ("C", C, 6), ("T", T, 15)):
        poly, err = mp.chebyfit(fn, [0, s_max], deg + 1, error=True)
        coeffs = [d(c) for c in poly]            # highest degree first
        print(f"// {name}: degree {deg} in s = r^2, Chebyshev fit error {mp.nstr(err, 5)}")
        print(f"constexpr double k{name}[{deg + 1}] = {{" +
              ", ".join(c.hex() for c in coeffs) + "};")


if __name__ == "__main__" and len(__import__("sys").argv) == 1:
    main()


def fit_small(rmax=0.2, deg_s=3, deg_c=3):
    """Small-angle sin/cos for the heading rotation recurrence (|d| <= rmax):
        sin(d) = d + d^3 * Ps(d^2),  cos(d) - 1 = -d^2/2 + d^4 * Pc(d^2)."""
    smax = mp.mpf(rmax) ** 2

    def Ps(s):
        if s == 0:
            return -mp.mpf(1) / 6
        r = mp.sqrt(s)
        return (mp.sin(r) - r) / (r * s)

    def Pc(s):
        if s == 0:
            return mp.mpf(1) / 24
        r = mp.sqrt(s)
        return (mp.cos(r) - 1 + s / 2) / (s * s)

    for name, fn, deg in (("RS", Ps, deg_s), ("RC", Pc, deg_c)):
        poly, err = mp.chebyfit(fn, [0, smax], deg + 1, error=True)
        print(f"// {name}: degree {deg} in d^2 on |d| <= {rmax}, fit error {mp.nstr(err, 5)}")
        print(f"constexpr double k{name}[{deg + 1}] = {{" +
              ", ".join(d(c).hex() for c in poly) + "};")


if __name__ == "__main__" and "--small" in __import__("sys").argv:
    fit_small()


def fit_tan_rational(xmax=1.1, m=3, n=4, iters=40, nodes=240, monic=False):
    """Rational tan for the steering angle, no range reduction (|x| <= xmax):
        tan(x) = x + x^3 * P(x^2) / Q(x^2),   Q(0) = 1.
    Linearised least squares (Sanathanan-Koerner) with Lawson weights for a
    near-minimax relative error of P/Q against T(s) = (tan(r) - r) / r^3.
    monic: P and Q divided by Q's leading coefficient before rounding (the
    first Horner step of Q is then an add: no constant-bus move).
    The shipped kTP/kTQ: --tan-rational --monic (m = n = 3)."""
    mp.mp.dps = 60
    smax = mp.mpf(xmax) ** 2

    def T(s):
        if s == 0:
            return mp.mpf(1) / 3
        r = mp.sqrt(s)
        return (mp.tan(r) - r) / (r * s)

    pts = [smax * (1 - mp.cos(mp.pi * (k + mp.mpf(1) / 2) / nodes)) / 2 for k in range(nodes)]
    fv = [T(s) for s in pts]
    w = [mp.mpf(1)] * nodes
    qprev = [mp.mpf(1)] * nodes
    for it in range(iters):
        rows, rhs = [], []
        for s, f, wi, qp in zip(pts, fv, w, qprev):
            sc = mp.sqrt(wi) / (qp * f)
            rows.append([sc * s ** i for i in range(m + 1)] +
                        [-sc * f * s ** j for j in range(1, n + 1)])
            rhs.append(sc * f)
        x = mp.qr_solve(mp.matrix(rows), mp.matrix(rhs))[0]
        p = [x[i] for i in range(m + 1)]
        q = [mp.mpf(1)] + [x[m + 1 + j] for j in range(n)]

        def R(s):
            return mp.polyval(p[::-1], s) / mp.polyval(q[::-1], s)

        err = [(R(s) - f) / f for s, f in zip(pts, fv)]
        qprev = [mp.polyval(q[::-1], s) for s in pts]
        if it >= 5:
            tot = sum(wi * abs(e) for wi, e in zip(w, err))
            w = [wi * abs(e) / tot * nodes for wi, e in zip(w, err)]
    if monic:
        p = [c / q[-1] for c in p]
        q = [c / q[-1] for c in q]
    pd = [mp.mpf(d(c)) for c in p]
    qd = [mp.mpf(d(c)) for c in q]

    def Rd(s):
        return mp.polyval(pd[::-1], s) / mp.polyval(qd[::-1], s)

    worst = max(abs((Rd(s) - T(s)) / T(s)) for s in (smax * k / 2000 for k in range(2001)))
    print(f"// tan(x) = x + x^3 * TP(x^2) / TQ(x^2) on |x| <= {xmax}, rel. error of P/Q "
          f"{mp.nstr(worst, 5)}")
    print(f"constexpr double kTP[{m + 1}] = {{" + ", ".join(d(c).hex() for c in p[::-1]) + "};")
    print(f"constexpr double kTQ[{n + 1}] = {{" + ", ".join(d(c).hex() for c in q[::-1]) + "};")


if __name__ == "__main__" and "--tan-rational" in __import__("sys").argv:
    if "--monic" in __import__("sys").argv:
        fit_tan_rational(m=3, n=3, monic=True)
    else:
        fit_tan_rational()


def two_over_pi_words(n=38):
    """2/pi as n big-endian 32-bit words of its binary fraction (the
    Payne-Hanek table of mpc_trig.h, kTwoOverPiBits)."""
    mp.mp.prec = 32 * n + 64
    v = int(mp.floor(2 / mp.pi * mp.mpf(2) ** (32 * n)))
    return [(v >> (32 * (n - 1 - i))) & 0xffffffff for i in range(n)]


if __name__ == "__main__" and "--two-over-pi" in __import__("sys").argv:
    print(", ".join("0x%08x" % w for w in two_over_pi_words()))
