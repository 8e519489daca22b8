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


if __name__ == "__main__" and "--small" not in __import__("sys").argv:
    main()


def fit_small(rmax=0.25, deg_s=4, deg_c=4):
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
