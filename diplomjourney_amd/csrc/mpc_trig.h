// mpc_trig.h — fp64 tan and sincos for the MPC step, written for gfx950's VALU.
//
// Why not the device library's tan(): on gfx950 it evaluates the Payne-Hanek
// large-argument reduction unconditionally (both reductions are computed and
// one is selected), ~70 of its ~155 instructions per call, although the
// kernel's arguments are steering angles (|beta| <= 1.05) and headings.
// Here the reduction is a branch-free 3-part Cody-Waite (pi/2 = P1+P2+P3, P1
// and P2 with 33 significant bits, so k*P1 and k*P2 are exact for |k| <= 2^19)
// producing a double-double remainder, followed by near-minimax polynomials on
// |r| <= pi/4 (coefficients from tools/fit_trig.py, mpmath).  Arguments beyond
// the Cody-Waite range take a (wave-divergent, in practice never taken) branch
// to an integer Payne-Hanek reduction (reduce_pio2_large), so results are
// correct for every input without the device library's large-argument code.
//
// Accuracy: faithful (< 1 ulp); see tests/test_trig.py for the measured error
// against mpmath and the agreement rate with glibc (which the reference uses).
// The same source compiles for the host, where it is tested bit for bit
// against the device build.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define MPC_HD __host__ __device__
#else
#define MPC_HD
#endif

namespace mpc {
namespace trig {

// Cody-Waite pi/2 = P1 + P2 + P3 (tools/fit_trig.py)
constexpr double kP1 = 0x1.921fb54400000p+0;
constexpr double kP2 = 0x1.0b4611a600000p-34;
constexpr double kP3 = 0x1.3198a2e037073p-69;
constexpr double kTwoOverPi = 0x1.45f306dc9c883p-1;
// |x| <= kFastMax  =>  |k| <= 2^19
constexpr double kFastMax = 0x1p19 * 1.5707963267948966;

// sin(r) = r + r^3 * S(r^2);  S[6] = -1/6          (highest degree first)
constexpr double kS[7] = {-0x1.ab17d393166dcp-41, 0x1.61217f0abf087p-33, -0x1.ae645412c46d3p-26,
                          0x1.71de3a5460952p-19,  -0x1.a01a01a019938p-13, 0x1.1111111111110p-7,
                          -0x1.5555555555555p-3};
// cos(r) = 1 - r^2/2 + r^4 * C(r^2);  C[6] = 1/24
constexpr double kC[7] = {0x1.ab785a9b7d08fp-45,  -0x1.9394ba0c2b394p-37, 0x1.1eed8deb973d2p-29,
                          -0x1.27e4fb7712d61p-22, 0x1.a01a01a019d0ap-16,  -0x1.6c16c16c16c16p-10,
                          0x1.5555555555555p-5};
// tan(r) = r + r^3 * T(r^2);  T[15] = 1/3
constexpr double kT[16] = {0x1.090dd50c4e26cp-18, -0x1.46ffa51d98a1ep-17, 0x1.47c7055045e77p-16,
                           -0x1.562bc1c9b4034p-17, 0x1.c6cf3cb6be147p-16, 0x1.1c9d930b42224p-15,
                           0x1.9e442bd4b147bp-14,  0x1.f4827710891adp-13, 0x1.35639727a6c93p-11,
                           0x1.7da2a66dc0210p-10,  0x1.d6d3d9596ac82p-9,  0x1.226e353ec9951p-7,
                           0x1.664f48834f976p-6,   0x1.ba1ba1ba1a515p-5,  0x1.111111111111bp-3,
                           0x1.5555555555555p-2};

// fma(a, b, c) with c a compile-time coefficient.  On gfx950 hipcc selects
// the two-address v_fmac_f64 for a Horner step and then has to copy the
// (loop-invariant) coefficient into the accumulator first: two VALU ops and
// two VGPRs per coefficient.  The three-address VOP3 form with the
// coefficient in an SGPR pair is one VALU op and no VGPRs.
MPC_HD inline double fma_k(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
#else
  return fma(a, b, c);
#endif
}

// `lead` is c[0].  Horner's first step fma(c0, z, c1) has two coefficient
// operands, and gfx9 VALU instructions read at most one SGPR, so c0 has to be
// in a VGPR: hipcc re-materialises it with a v_mov per evaluation unless the
// caller passes a copy it keeps resident (see Leads).
template <int N>
MPC_HD inline double horner(const double (&c)[N], double z, int skip_last = 0,
                            double lead = 0.0, bool have_lead = false) {
  double p = have_lead ? lead : c[0];
#pragma unroll
  for (int i = 1; i < N; ++i)
    if (i < N - skip_last) p = fma_k(p, z, c[i]);
  return p;
}

// x = k*pi/2 + (hi + lo), |hi| <= pi/4 (+ulps); exact-ish double-double.
struct Reduced {
  double hi, lo;
  int q;
};

MPC_HD inline Reduced reduce_pio2(double x) {
  // + 0.0 turns rint's -0 into +0, so x = -0 reduces to hi = -0 (sin(-0) = -0)
  const double k = rint(x * kTwoOverPi) + 0.0;
  double r = fma(-k, kP1, x);  // exact: k*P1 exact, x and k*P1 within a factor 2
  double w = k * kP2;          // exact
  const double t = r;
  r = t - w;
  w = fma(k, kP3, -((t - r) - w));
  Reduced o;
  o.hi = r - w;
  o.lo = (r - o.hi) - w;
  o.q = static_cast<int>(k);
  return o;
}

// sin / cos of hi + lo, |hi| <= pi/4
MPC_HD inline double ksin(double x, double y) {
  const double z = x * x;
  const double v = z * x;
  const double r = horner(kS, z, 1);  // S1 + z*(S2 + ...)
  return x - ((z * (0.5 * y - v * r) - y) - v * kS[6]);
}

MPC_HD inline double kcos(double x, double y) {
  const double z = x * x;
  const double r = z * horner(kC, z);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

// 1/d for |d| in [2^-60, 2]: hardware reciprocal estimate + two Newton steps
// (relative error ~2^-100 before the final rounding).
MPC_HD inline double recip(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(d);
#else
  double r = 1.0 / d;
#endif
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

// tan (odd == 0) or -1/tan (odd == 1) of hi + lo, |hi| <= pi/4.  Branch-free:
// both quadrant forms are formed and one is selected per lane.
MPC_HD inline double ktan(double x, double y, bool odd) {
  const double z = x * x;
  const double u = (x * z) * horner(kT, z);
  const double th = x + u;
  double tl = (x - th) + u;               // exact error of th (|x| >= |u|)
  tl = fma(y, fma(th, th, 1.0), tl);      // + lo * sec^2
  const double a = -recip(th);            // -1/th
  const double e = fma(a, th, 1.0) + a * tl;  // 1 + a*(th + tl)
  const double cot = fma(a, e, a);
  return odd ? cot : th + tl;
}

// Steering-angle tangent without range reduction, |x| <= kTanMax:
//   tan(x) = x + x^3 * TP(x^2) / TQ(x^2)
// (tools/fit_trig.py --tan-rational --monic: degrees 3/3, rel. error of P/Q
// 6.2e-17 with the rounded coefficients).  TQ is monic, so its first Horner
// step is an add (no constant-bus move for a second coefficient operand).
// One reciprocal estimate and one Newton step form 1/Q; P * (1/Q) is not
// corrected further (its rounding enters tan with weight x^3 R / tan <= 0.44).
// The estimate (v_rcp_f64) is good to 2^-24.4 and one Newton step leaves the
// reciprocal off its rounded value on ~40 % of mantissas
// (tools/micro/rcp_acc.hip), so the host build reproduces the device bits only
// with the device's own estimates: rcp_estimate() reads them from a table a
// test installs (g_host_rcp_estimate, tests/replica_harness.cpp; the estimates
// come from the device through mpc_rcp_estimate).  Without a table the host
// build uses 1.0 / q (the CPU-side tests compare it within tolerances).
// ~14 VALU instead of the ~50 of a Cody-Waite reduction and the
// quadrant/cotangent reconstruction of tan_core.  The steering bound of the
// reference's config is 60 deg = 1.047 rad; a larger |beta| makes the
// candidate irregular (recomputed with tan_fast).
constexpr double kTanMax = 1.1;
constexpr double kTP[4] = {0x1.2806dd56192d1p-14, -0x1.e9a6933b8c31cp-1, 0x1.4e67ddcc55034p+6,
                           -0x1.44bcc514568d3p+10};
constexpr double kTQ[4] = {0x1.0000000000000p+0, -0x1.7f12a2265b864p+6, 0x1.c462cc7b84963p+10,
                           -0x1.e71b279e81d3cp+11};   // Q in [-3893, -1530] on |x| <= 1.1

#if !defined(__HIP_DEVICE_COMPILE__)
inline double (*g_host_rcp_estimate)(double) = nullptr;
#endif

// The hardware reciprocal estimate (device), or its host stand-in.
MPC_HD inline double rcp_estimate(double q) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcp(q);
#else
  return g_host_rcp_estimate ? g_host_rcp_estimate(q) : 1.0 / q;
#endif
}

// Leading polynomial coefficients of the hot loop's trig, held in VGPRs by
// the rollout kernel (one copy per lane instead of a v_mov per use); equal to
// the constants, so results are bitwise those of the default arguments.
struct Leads {
  double tp, rs, rc;
};

// tan_small's denominator Q(s), s = x^2 (monic: the first step is an add).
MPC_HD inline double tan_small_q(double s) {
  double q = s + kTQ[1];
  q = fma_k(q, s, kTQ[2]);
  return fma_k(q, s, kTQ[3]);
}

MPC_HD inline double tan_small(double x, const Leads* ld = nullptr) {
  const double s = x * x;
  const double p = ld ? horner(kTP, s, 0, ld->tp, true) : horner(kTP, s);
  const double q = tan_small_q(s);
  double r = rcp_estimate(q);
  r = fma(r, fma(-q, r, 1.0), r);
  return fma(x * s, p * r, x);
}

// Core forms: valid for |x| <= kFastMax only (the caller guarantees it or
// flags the argument as irregular and recomputes with the full forms below).
MPC_HD inline double tan_core(double x) {
  const Reduced r = reduce_pio2(x);
  const double t = ktan(r.hi, r.lo, (r.q & 1) != 0);
  return x == 0.0 ? x : t;  // tan(+-0) = +-0
}

MPC_HD inline void sincos_reduced(const Reduced& r, double* s, double* c);

MPC_HD inline void sincos_core(double x, double* s, double* c) {
  sincos_reduced(reduce_pio2(x), s, c);
}

// ---------------------------------------------------------------------------
// Payne-Hanek reduction for |x| > kFastMax (up to DBL_MAX), in integer
// arithmetic.  It replaces the device library's large-argument path, whose
// inlined code set the VGPR budget of every kernel that can meet such an
// argument (the rollout kernel's irregular-candidate recompute: 121 VGPRs
// with it, ~92 without), and it is the same code on the host.
//
// x = m * 2^e (m the 53-bit significand).  With 2/pi = sum_i W[i] 2^-32(i+1)
// (kTwoOverPiBits, tools/fit_trig.py --two-over-pi), the words with
// e - 32(i+1) >= 2 only add multiples of 4 to x*2/pi and are skipped; the next
// eight words (256 bits) give x*2/pi mod 4 with an absolute error below
// 2^-138, i.e. 2^-77 relative to the smallest reduced argument a double can
// produce (~2^-61).  Two leading zero words let the window start before the
// binary point (e >= -33 here).
constexpr uint32_t kTwoOverPiBits[40] = {
    0x00000000, 0x00000000, 0xa2f9836e, 0x4e441529, 0xfc2757d1, 0xf534ddc0,
    0xdb629599, 0x3c439041, 0xfe5163ab, 0xdebbc561, 0xb7246e3a, 0x424dd2e0,
    0x06492eea, 0x09d1921c, 0xfe1deb1c, 0xb129a73e, 0xe88235f5, 0x2ebb4484,
    0xe99c7026, 0xb45f7e41, 0x3991d639, 0x835339f4, 0x9c845f8b, 0xbdf9283b,
    0x1ff897ff, 0xde05980f, 0xef2f118b, 0x5a0a6d1f, 0x6d367ecf, 0x27cb09b7,
    0x4f463f66, 0x9e5fea2d, 0x7527bac7, 0xebe5f17b, 0x3d0739f7, 0x8a5292ea,
    0x6bfb5fb1, 0x1f8d5d08, 0x56033046, 0xfc7b6bab,
};

MPC_HD inline void umul64wide(uint64_t a, uint64_t b, uint64_t& hi, uint64_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  hi = __umul64hi(a, b);
  lo = a * b;
#else
  const unsigned __int128 p = static_cast<unsigned __int128>(a) * b;
  hi = static_cast<uint64_t>(p >> 64);
  lo = static_cast<uint64_t>(p);
#endif
}

// x finite, |x| > kFastMax: x = q*pi/2 + (hi + lo), |hi + lo| <= pi/4.
MPC_HD inline Reduced reduce_pio2_large(double x) {
  uint64_t bits;
  __builtin_memcpy(&bits, &x, 8);
  const bool neg = (bits >> 63) != 0;
  const int e = static_cast<int>((bits >> 52) & 0x7ff) - 1075;          // x = m * 2^e
  const uint64_t m = (bits & 0x000fffffffffffffull) | 0x0010000000000000ull;
  const int i0 = ((e + 30) >> 5) + 1;               // first word used (+2: the zero words)
  auto w64 = [&](int k) {
    return (static_cast<uint64_t>(kTwoOverPiBits[i0 + 2 * k]) << 32) |
           kTwoOverPiBits[i0 + 2 * k + 1];
  };
  // P = m * (w0 w1 w2 w3): limbs R1 (bits 192..255), R2, R3 (bits 64..127);
  // the binary point of x*2/pi sits at bit 32*(i0-2+8) - e of P, in [223, 255).
  uint64_t h0, l0, h1, l1, h2, l2, h3, l3;
  umul64wide(m, w64(0), h0, l0);
  umul64wide(m, w64(1), h1, l1);
  umul64wide(m, w64(2), h2, l2);
  umul64wide(m, w64(3), h3, l3);
  (void)h0;
  (void)l3;
  const uint64_t R3 = h3 + l2;
  const uint64_t c3 = R3 < l2 ? 1 : 0;
  uint64_t R2 = h2 + l1;
  uint64_t c2 = R2 < l1 ? 1 : 0;
  R2 += c3;
  c2 += (R2 < c3) ? 1 : 0;
  const uint64_t R1 = h1 + l0 + c2;
  const int t = 32 * (i0 + 6) - e - 192;            // binary point at bit 192 + t, t in [31, 63)
  const uint64_t F_hi = (R2 >> t) | (R1 << (64 - t));   // the 128 fraction bits
  const uint64_t F_lo = (R3 >> t) | (R2 << (64 - t));
  int q = static_cast<int>((R1 >> t) & 3);
  // fraction f in [0, 1) -> [-1/2, 1/2): above 1/2 take f - 1 and q + 1
  double fh, fl;
  const double k2m64 = 0x1p-64;
  if (F_hi >> 63) {
    const uint64_t nlo = ~F_lo + 1;                 // 2^128 - F
    const uint64_t nhi = ~F_hi + (nlo == 0 ? 1 : 0);
    q += 1;
    const double a = static_cast<double>(nhi);      // rounded; the rest is exact below
    const uint64_t ai = static_cast<uint64_t>(a);
    const double r = static_cast<double>(static_cast<int64_t>(nhi - ai)) +
                     static_cast<double>(nlo) * k2m64;
    fh = -(a * k2m64);
    fl = -(r * k2m64);
  } else {
    const double a = static_cast<double>(F_hi);
    const uint64_t ai = static_cast<uint64_t>(a);
    const double r = static_cast<double>(static_cast<int64_t>(F_hi - ai)) +
                     static_cast<double>(F_lo) * k2m64;
    fh = a * k2m64;
    fl = r * k2m64;
  }
  const double s0 = fh + fl;                        // normalise the fraction
  fl = fl - (s0 - fh);
  fh = s0;
  // (fh + fl) * pi/2 in double-double
  constexpr double kPio2Hi = 0x1.921fb54442d18p+0, kPio2Lo = 0x1.1a62633145c07p-54;
  const double ph = fh * kPio2Hi;
  const double pl = fma(fh, kPio2Hi, -ph) + (fh * kPio2Lo + fl * kPio2Hi);
  Reduced o;
  o.hi = ph + pl;
  o.lo = pl - (o.hi - ph);
  o.q = q;
  if (neg) {
    o.hi = -o.hi;
    o.lo = -o.lo;
    o.q = -q;
  }
  return o;
}

// Full forms: any argument.  |x| <= kFastMax: the Cody-Waite cores; larger
// finite x: Payne-Hanek; inf / NaN: NaN.
MPC_HD inline double tan_fast(double x) {
  if (fabs(x) <= kFastMax) return tan_core(x);
  if (!(fabs(x) < __builtin_inf())) return x - x;
  const Reduced r = reduce_pio2_large(x);
  return ktan(r.hi, r.lo, (r.q & 1) != 0);
}

MPC_HD inline void sincos_reduced(const Reduced& r, double* s, double* c) {
  const double sn = ksin(r.hi, r.lo);
  const double cs = kcos(r.hi, r.lo);
  const int q = r.q & 3;
  double S = (q & 1) ? cs : sn;
  double C = (q & 1) ? sn : cs;
  if (q & 2) S = -S;
  if ((q + 1) & 2) C = -C;
  *s = S;
  *c = C;
}

MPC_HD inline void sincos_fast(double x, double* s, double* c) {
  if (fabs(x) <= kFastMax) {
    sincos_core(x, s, c);
    return;
  }
  if (!(fabs(x) < __builtin_inf())) {
    *s = *c = x - x;
    return;
  }
  sincos_reduced(reduce_pio2_large(x), s, c);
}

// ---------------------------------------------------------------------------
// Heading rotation (MPC_HEADING_ROTATE mode).  The heading advances by a small
// increment each step (|dphi| <= v_max/L * tan(beta_max) * dt = 0.173 rad in
// the reference's config), so (sin phi, cos phi) can be carried along the
// rollout and rotated by dphi instead of re-evaluated with a full range
// reduction:  s' = s + (s*cm1 + c*sd),  c' = c + (c*cm1 - s*sd)  with
// sd = sin(dphi), cm1 = cos(dphi) - 1 from short polynomials on |d| <= 0.2
// (tools/fit_trig.py --small).
constexpr double kRotMax = 0.2;
// sin(d) = d + d^3 * RS(d^2);  RS[3] ~ -1/6   (near-minimax on |d| <= 0.2; the
// abs. error of the d^3 term is <= 4e-18, 0.15 ulp of sin(0.2))
constexpr double kRS[4] = {0x1.719963b18b037p-19, -0x1.a019fabe07951p-13, 0x1.11111110d8aedp-7,
                           -0x1.5555555555543p-3};
// cos(d) - 1 = -d^2/2 + d^4 * RC(d^2);  RC[3] ~ 1/24   (abs. error <= 7e-20)
constexpr double kRC[4] = {-0x1.27b71672cf54cp-22, 0x1.a019fd094f3a7p-16, -0x1.6c16c16bf129ep-10,
                           0x1.555555555554fp-5};

// sd = sin(d), cm1 = cos(d) - 1 for |d| <= kRotMax (larger increments make
// the candidate irregular: it is recomputed with direct evaluation)
// cm1 = z * (-1/2 + z * RC(z)): the -1/2 enters as an fma addend (inline
// constant), one multiply fewer than -z/2 + z^2 * RC(z); its rounding of
// -1/2 + z*RC adds at most 2^-54 relative, far below cm1's weight in c'.
// (The full tree's per-control factors, mpc_fulltree.h.)
MPC_HD inline void rotation_factors(double d, double& sd, double& cm1,
                                    const Leads* ld = nullptr) {
  const double z = d * d;
  sd = fma(d * z, ld ? horner(kRS, z, 0, ld->rs, true) : horner(kRS, z), d);
  cm1 = z * fma(z, ld ? horner(kRC, z, 0, ld->rc, true) : horner(kRC, z), -0.5);
}

// (s, c) <- rotation of (s, c) by the angle whose factors are (sd, cm1)
MPC_HD inline void rotate_by(double sd, double cm1, double& s, double& c) {
  const double s1 = s + fma(c, sd, s * cm1);
  const double c1 = c + fma(-s, sd, c * cm1);
  s = s1;
  c = c1;
}

// The candidate rollout's form: sd = sin(d) and cd = cos(d) itself, cd =
// 1 + z * (-1/2 + z * RC(z)) (same operation count as cm1, the final multiply
// becomes an fma with the inline constant 1), and the rotation as a plain
// complex product, s' = s*cd + c*sd, c' = c*cd - s*sd: 4 VALU instead of 6.
// cd's rounding (<= 2^-53 absolute) costs about one ulp of (s, c) per step,
// ~1e-15 relative over the horizon; the rollout's results are pinned by its
// host replica (same functions) and against the oracle within 1e-13.
MPC_HD inline void rotation_sc(double d, double& sd, double& cd, const Leads* ld = nullptr) {
  const double z = d * d;
  sd = fma(d * z, ld ? horner(kRS, z, 0, ld->rs, true) : horner(kRS, z), d);
  cd = fma(z, fma(z, ld ? horner(kRC, z, 0, ld->rc, true) : horner(kRC, z), -0.5), 1.0);
}

MPC_HD inline void rotate_sc(double sd, double cd, double& s, double& c) {
  const double s1 = fma(c, sd, s * cd);
  const double c1 = fma(-s, sd, c * cd);
  s = s1;
  c = c1;
}

MPC_HD inline Leads const_leads() { return Leads{kTP[0], kRS[0], kRC[0]}; }

}  // namespace trig
}  // namespace mpc
