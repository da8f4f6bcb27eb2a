// farms_libm.h — correctly rounded atan2 / sin / cos for the FARMS_Flow path.
//
// The reference evaluates atan2, cos and sin with glibc (vFlow.cpp:325, 366,
// 1007-1008, 1120-1121, 1375-1377).  glibc 2.35's double versions round
// correctly on all but a vanishing fraction of arguments; ROCm's ocml versions
// are faithful (<= 1 ulp) and differ from glibc on ~30% of the local flows of a
// synthetic stream.  Since the validity gate, the window choice and the scale
// argmax are discontinuous, every such ulp is a potential record mismatch.
// These versions evaluate in double-double arithmetic (about 2^-100 relative
// error before the final rounding), so they return the correctly rounded
// result except on arguments within 2^-100 of a rounding boundary: bit-equal to
// glibc wherever glibc rounds correctly.  Only +, -, *, / and fma are used,
// so host and device builds return identical bits (compile with
// -ffp-contract=off).  tests/test_libm.py checks them against the host glibc.
//
// Domain: atan2 everywhere (IEEE special cases included); sin / cos for
// |x| < 2^26, NaN beyond (the path evaluates them only on atan2 results,
// |x| <= pi).  Compiler builtins only, so every function is host + device.
#ifndef FARMS_LIBM_H
#define FARMS_LIBM_H

#include <hip/hip_runtime.h>

namespace farms_libm {

// ---- constants (tools/gen_libm_tables.py: exact values split into doubles)
// pi/2 as three doubles, pi and pi/2 and pi/4 as double-doubles
constexpr double kPio2_1 = 0x1.921fb54442d18p+0, kPio2_2 = 0x1.1a62633145c07p-54, kPio2_3 = -0x1.f1976b7ed8fbcp-110;
constexpr double kPi_hi = 0x1.921fb54442d18p+1, kPi_lo = 0x1.1a62633145c07p-53;
constexpr double kPio2_hi = 0x1.921fb54442d18p+0, kPio2_lo = 0x1.1a62633145c07p-54;
constexpr double kPio4_hi = 0x1.921fb54442d18p-1, kPio4_lo = 0x1.1a62633145c07p-55;
constexpr double k3Pio4_hi = 0x1.2d97c7f3321d2p+1, k3Pio4_lo = 0x1.a79394c9e8a0ap-54;
constexpr double k2oPi = 0x1.45f306dc9c883p-1;
// atan(j/64), j = 0..64, {hi, lo}
constexpr double kAtanTab[65][2] = {
    {0x0.0p+0, 0x0.0p+0},
    {0x1.fff555bbb729bp-7, -0x1.220c39d4dff50p-61},
    {0x1.ffd55bba97625p-6, -0x1.5ec431444912cp-60},
    {0x1.7fb818430da2ap-5, -0x1.86ef8f794f105p-63},
    {0x1.ff55bb72cfdeap-5, -0x1.c934d86d23f1dp-60},
    {0x1.3f59f0e7c559dp-4, 0x1.ac4ce285df847p-58},
    {0x1.7ee182602f10fp-4, -0x1.cfb654c0c3d98p-58},
    {0x1.be39ebe6f07c3p-4, 0x1.f7b8f29a05987p-58},
    {0x1.fd5ba9aac2f6ep-4, -0x1.cd37686760c17p-59},
    {0x1.1e1fafb043727p-3, -0x1.b485914dacf8cp-59},
    {0x1.3d6eee8c6626cp-3, 0x1.61a3b0ce9281bp-57},
    {0x1.5c9811e3ec26ap-3, -0x1.054ab2c010f3dp-58},
    {0x1.7b97b4bce5b02p-3, 0x1.347b0b4f881cap-58},
    {0x1.9a6a8e96c8626p-3, 0x1.cf601e7b4348ep-59},
    {0x1.b90d7529260a2p-3, 0x1.17b10d2e0e5abp-61},
    {0x1.d77d5df205736p-3, 0x1.c648d1534597ep-57},
    {0x1.f5b75f92c80ddp-3, 0x1.8ab6e3cf7afbdp-57},
    {0x1.09dc597d86362p-2, 0x1.62e47390cb865p-56},
    {0x1.18bf5a30bf178p-2, 0x1.30ca4748b1bf9p-57},
    {0x1.278372057ef46p-2, -0x1.077cdd36dfc81p-56},
    {0x1.362773707ebccp-2, -0x1.963a544b672d8p-57},
    {0x1.44aa436c2af0ap-2, -0x1.5d5e43c55b3bap-56},
    {0x1.530ad9951cd4ap-2, -0x1.2566480884082p-57},
    {0x1.614840309cfe2p-2, -0x1.a725715711f00p-56},
    {0x1.6f61941e4def1p-2, -0x1.c63aae6f6e918p-56},
    {0x1.7d5604b63b3f7p-2, 0x1.69c885c2b249ap-56},
    {0x1.8b24d394a1b25p-2, 0x1.b6d0ba3748fa8p-56},
    {0x1.98cd5454d6b18p-2, 0x1.9e6c988fd0a77p-56},
    {0x1.a64eec3cc23fdp-2, -0x1.24dec1b50b7ffp-56},
    {0x1.b3a911da65c6cp-2, 0x1.ae187b1ca5040p-56},
    {0x1.c0db4c94ec9f0p-2, -0x1.cc1ce70934c34p-56},
    {0x1.cde53432c1351p-2, -0x1.a2cfa4418f1adp-56},
    {0x1.dac670561bb4fp-2, 0x1.a2b7f222f65e2p-56},
    {0x1.e77eb7f175a34p-2, 0x1.0e53dc1bf3435p-56},
    {0x1.f40dd0b541418p-2, -0x1.a3992dc382a23p-57},
    {0x1.0039c73c1a40cp-1, -0x1.b32c949c9d593p-55},
    {0x1.0657e94db30d0p-1, -0x1.d5b495f6349e6p-56},
    {0x1.0c6145b5b43dap-1, 0x1.974fa13b5404fp-58},
    {0x1.1255d9bfbd2a9p-1, -0x1.2bdaee1c0ee35p-58},
    {0x1.1835a88be7c13p-1, 0x1.c621cec00c301p-55},
    {0x1.1e00babdefeb4p-1, -0x1.928df287a668fp-58},
    {0x1.23b71e2cc9e6ap-1, 0x1.c421c9f38224ep-57},
    {0x1.2958e59308e31p-1, -0x1.09e73b0c6c087p-56},
    {0x1.2ee628406cbcap-1, 0x1.c5d5e9ff0cf8dp-55},
    {0x1.345f01cce37bbp-1, 0x1.1021137c71102p-55},
    {0x1.39c391cd4171ap-1, -0x1.2304331d8bf46p-55},
    {0x1.3f13fb89e96f4p-1, 0x1.ecf8b492644f0p-56},
    {0x1.445065b795b56p-1, -0x1.f76d0163f79c8p-56},
    {0x1.4978fa3269ee1p-1, 0x1.2419a87f2a458p-56},
    {0x1.4e8de5bb6ec04p-1, 0x1.4a33dbeb3796cp-55},
    {0x1.538f57b89061fp-1, -0x1.1bb74abda520cp-55},
    {0x1.587d81f732fbbp-1, -0x1.5e5c9d8c5a950p-56},
    {0x1.5d58987169b18p-1, 0x1.0028e4bc5e7cap-57},
    {0x1.6220d115d7b8ep-1, -0x1.2b785350ee8c1p-57},
    {0x1.66d663923e087p-1, -0x1.6ea6febe8bbbap-56},
    {0x1.6b798920b3d99p-1, -0x1.a80386188c50ep-55},
    {0x1.700a7c5784634p-1, -0x1.8c34d25aadef6p-56},
    {0x1.748978fba8e0fp-1, 0x1.7b2a6165884a1p-59},
    {0x1.78f6bbd5d315ep-1, 0x1.406a089803740p-55},
    {0x1.7d528289fa093p-1, 0x1.560821e2f3aa9p-55},
    {0x1.819d0b7158a4dp-1, -0x1.bf76229d3b917p-56},
    {0x1.85d69576cc2c5p-1, 0x1.6b66e7fc8b8c3p-57},
    {0x1.89ff5ff57f1f8p-1, -0x1.55b9a5e177a1bp-55},
    {0x1.8e17aa99cc05ep-1, -0x1.ec182ab042f61p-56},
    {0x1.921fb54442d18p-1, 0x1.1a62633145c07p-55},
};
// sin: (-1)^n / (2n+1)!, n = 0..14; cos: (-1)^n / (2n)!, n = 0..14
constexpr double kSinC[15][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.5555555555555p-3, -0x1.5555555555555p-57},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63},
    {-0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
    {-0x1.ae64567f544e4p-26, 0x1.c062e06d1f209p-80},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
    {-0x1.ae7f3e733b81fp-41, -0x1.1d8656b0ee8cbp-97},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},
    {-0x1.2f49b46814157p-57, -0x1.2650f61dbdcb4p-112},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},
    {-0x1.761b41316381ap-75, 0x1.3423c7d91404fp-130},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},
    {-0x1.d1ab1c2dccea3p-94, -0x1.054d0c78aea14p-149},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157},
};
constexpr double kCosC[15][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.0000000000000p-1, 0x0.0p+0},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59},
    {-0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
    {-0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
    {-0x1.93974a8c07c9dp-37, -0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
    {-0x1.6827863b97d97p-53, -0x1.eec01221a8b0bp-107},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
    {-0x1.0ce396db7f853p-70, 0x1.aebcdbd20331cp-124},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},
    {-0x1.88e85fc6a4e5ap-89, 0x1.71c37ebd16540p-143},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},
};
// atan: (-1)^n / (2n+1), n = 0..9
constexpr double kAtanC[10][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},
    {-0x1.5555555555555p-2, -0x1.5555555555555p-56},
    {0x1.999999999999ap-3, -0x1.999999999999ap-57},
    {-0x1.2492492492492p-3, -0x1.2492492492492p-57},
    {0x1.c71c71c71c71cp-4, 0x1.c71c71c71c71cp-58},
    {-0x1.745d1745d1746p-4, 0x1.745d1745d1746p-59},
    {0x1.3b13b13b13b14p-4, -0x1.3b13b13b13b14p-58},
    {-0x1.1111111111111p-4, -0x1.1111111111111p-60},
    {0x1.e1e1e1e1e1e1ep-5, 0x1.e1e1e1e1e1e1ep-61},
    {-0x1.af286bca1af28p-5, -0x1.af286bca1af28p-59},
};

// ---- double-double arithmetic (hi + lo, |lo| <= ulp(hi) / 2)
struct dd {
    double hi, lo;
};

__host__ __device__ inline dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd fast_two_sum(double a, double b) {  // |a| >= |b| or a == 0
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd two_prod(double a, double b) {
    const double p = a * b;
    return {p, __builtin_fma(a, b, -p)};
}
__host__ __device__ inline dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
__host__ __device__ inline dd dd_add(dd a, dd b) {  // accurate addition (relative error ~2^-105)
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fast_two_sum(s.hi, s.lo);
}
__host__ __device__ inline dd dd_add_d(dd a, double b) {
    dd s = two_sum(a.hi, b);
    s.lo += a.lo;
    return fast_two_sum(s.hi, s.lo);
}
__host__ __device__ inline dd dd_mul(dd a, dd b) {
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return fast_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd dd_mul_d(dd a, double b) {
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return fast_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd dd_div(dd a, dd b) {  // three quotient digits
    const double q1 = a.hi / b.hi;
    dd r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
    const double q2 = r.hi / b.hi;
    r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
    const double q3 = r.hi / b.hi;
    return dd_add_d(fast_two_sum(q1, q2), q3);
}
__host__ __device__ inline dd dd_c(const double (&c)[2]) { return {c[0], c[1]}; }

// ---- sin / cos
// x = q * pi/2 + r, |r| <= pi/4 (+ rounding of q), r as a double-double: pi/2
// in three parts, each product with q exact or negligible.
__host__ __device__ inline dd reduce_pio2(double x, int &q) {
    const double kd = __builtin_rint(x * k2oPi);
    q = (int)kd;
    if (q == 0) return {x, 0.0};
    dd r = dd_add_d(dd_neg(two_prod(kd, kPio2_1)), x);
    r = dd_add(r, dd_neg(two_prod(kd, kPio2_2)));
    return dd_add_d(r, -(kd * kPio2_3));
}
// Taylor series on |r| <= pi/4 (terms to r^29 / r^28: truncation < 2^-106)
__host__ __device__ inline dd sin_poly(dd r) {
    const dd z = dd_mul(r, r);
    dd s = dd_c(kSinC[14]);
    for (int n = 13; n >= 0; --n) s = dd_add(dd_mul(s, z), dd_c(kSinC[n]));
    return dd_mul(s, r);
}
__host__ __device__ inline dd cos_poly(dd r) {
    const dd z = dd_mul(r, r);
    dd s = dd_c(kCosC[14]);
    for (int n = 13; n >= 0; --n) s = dd_add(dd_mul(s, z), dd_c(kCosC[n]));
    return s;
}
// quadrant q of sin (cosine: q + 1)
__host__ __device__ inline double sin_quadrant(dd r, int q) {
    const dd v = (q & 1) ? cos_poly(r) : sin_poly(r);
    return (q & 2) ? -v.hi : v.hi;  // v.hi = RN(v.hi + v.lo): the normalised sum
}

__host__ __device__ inline double sin_dd(double x) {
    const double ax = __builtin_fabs(x);
    if (!(ax < 67108864.0)) return x - x + __builtin_nan("");  // NaN, inf, |x| >= 2^26: outside the domain
    if (ax < 0x1p-30) return x;              // sin x = x (1 - x^2/6): within half an ulp of x
    int q;
    const dd r = reduce_pio2(x, q);
    return sin_quadrant(r, q);
}

__host__ __device__ inline double cos_dd(double x) {
    const double ax = __builtin_fabs(x);
    if (!(ax < 67108864.0)) return x - x + __builtin_nan("");
    if (ax < 0x1p-30) return 1.0;  // cos x = 1 - x^2/2: within half an ulp of 1
    int q;
    const dd r = reduce_pio2(x, q);
    return sin_quadrant(r, q + 1);
}

// ---- atan2
// atan(t), t in [0, 1] as a double-double: atan(t) = atan(c) + atan(u) with
// c = j/64 nearest t and u = (t - c) / (1 + t c), |u| <= 2^-7 (series to u^19).
__host__ __device__ inline dd atan_01(dd t) {
    const int j = (int)__builtin_rint(t.hi * 64.0);
    const double c = (double)j * 0.015625;
    const dd num = dd_add_d(t, -c);
    const dd den = dd_add_d(dd_mul_d(t, c), 1.0);
    const dd u = dd_div(num, den);
    const dd z = dd_mul(u, u);
    dd s = dd_c(kAtanC[9]);
    for (int n = 8; n >= 0; --n) s = dd_add(dd_mul(s, z), dd_c(kAtanC[n]));
    return dd_add(dd_c(kAtanTab[j]), dd_mul(s, u));
}

__host__ __device__ inline double atan2_dd(double y, double x) {
    if (x != x || y != y) return x + y;
    const bool xneg = __builtin_signbit(x);
    const double ax = __builtin_fabs(x), ay = __builtin_fabs(y);
    const double inf = __builtin_inf();
    double res;
    if (ay == 0.0) res = xneg ? kPi_hi : 0.0;  // atan2(+-0, x): +-0 or +-pi
    else if (ax == inf && ay == inf) res = xneg ? k3Pio4_hi : kPio4_hi;
    else if (ax == inf) res = xneg ? kPi_hi : 0.0;
    else if (ax == 0.0 || ay == inf) res = kPio2_hi;
    else {
        // t = min / max as a double-double (exact remainder by fma)
        const bool swap = ay > ax;
        const double n = swap ? ax : ay, d = swap ? ay : ax;
        const double qh = n / d;
        const dd t = fast_two_sum(qh, __builtin_fma(-qh, d, n) / d);
        dd a = atan_01(t);
        if (swap) a = dd_add(dd{kPio2_hi, kPio2_lo}, dd_neg(a));
        if (xneg) a = dd_add(dd{kPi_hi, kPi_lo}, dd_neg(a));
        res = a.hi;
    }
    return __builtin_copysign(res, y);
}

// ---- fast paths (Ziv): a cheaper evaluation with a proven error bound, and
// its result only where that bound decides the rounding; elsewhere (about one
// call in 2^12) the full double-double evaluation above.  Both round correctly,
// so the functions below return exactly what sin_dd / cos_dd / atan2_dd do.
//
// round_ok: v = hi + lo (normalised) approximates the true value t with
// |t - v| < eps * |hi|; RN(t) = hi iff both ends of that interval round to hi
// (rounding is monotone).  kFastEps leaves a factor >= 8 over the evaluation
// errors derived below.
constexpr double kFastEps = 0x1p-66;
#ifndef FARMS_LIBM_FALLBACK
#define FARMS_LIBM_FALLBACK() ((void)0)  // host check builds count the full evaluations here
#endif
__host__ __device__ inline bool round_ok(dd v) {
    const double e = kFastEps * __builtin_fabs(v.hi);
    return v.hi + (v.lo + e) == v.hi && v.hi + (v.lo - e) == v.hi;
}
// sin(r) = r (1 + u) and cos(r) = 1 + u' on |r| <= pi/4 + 2^-50, z = r^2 <= 0.62:
// the Taylor terms n >= 4 in double (Horner on z.hi; truncation after n = 9
// below z^10 / 21! < 2^-72 relative; rounding < 2^-69 of the result, these
// terms being < 2.2e-6 / 2.5e-5 of it), n = 1..3 in double-double.
__host__ __device__ inline dd sin_poly_fast(dd r, dd z) {
    double t = kSinC[9][0];
    for (int n = 8; n >= 4; --n) t = __builtin_fma(t, z.hi, kSinC[n][0]);
    dd a = dd_add_d(dd_c(kSinC[3]), t * z.hi);             // S3 + z T
    a = dd_add(dd_c(kSinC[2]), dd_mul(a, z));              // S2 + z a
    a = dd_add(dd_c(kSinC[1]), dd_mul(a, z));              // S1 + z a
    return dd_add(r, dd_mul(r, dd_mul(a, z)));             // r + r z a
}
__host__ __device__ inline dd cos_poly_fast(dd z) {
    double t = kCosC[10][0];
    for (int n = 9; n >= 4; --n) t = __builtin_fma(t, z.hi, kCosC[n][0]);
    dd a = dd_add_d(dd_c(kCosC[3]), t * z.hi);
    a = dd_add(dd_c(kCosC[2]), dd_mul(a, z));
    a = dd_add(dd_c(kCosC[1]), dd_mul(a, z));
    return dd_add_d(dd_mul(a, z), 1.0);                    // 1 + z a
}
// sin and cos of x (|x| < 2^26), correctly rounded, one range reduction
__host__ __device__ inline void cr_sincos(double x, double *s, double *c) {
    const double ax = __builtin_fabs(x);
    if (!(ax < 67108864.0)) { *s = *c = x - x + __builtin_nan(""); return; }
    if (ax < 0x1p-30) { *s = x; *c = 1.0; return; }
    int q;
    const dd r = reduce_pio2(x, q);
    dd z = two_prod(r.hi, r.hi);
    z.lo += 2.0 * r.hi * r.lo;
    z = fast_two_sum(z.hi, z.lo);
    const dd ps = sin_poly_fast(r, z), pc = cos_poly_fast(z);
    // quadrant q: sin x = (+-) sin r or cos r, cos x likewise one quadrant on
    const dd vs = (q & 1) ? pc : ps, vc = (q & 1) ? ps : pc;
    const bool ok = round_ok(vs) && round_ok(vc);
    double sv = (q & 2) ? -vs.hi : vs.hi;
    double cv = ((q + 1) & 2) ? -vc.hi : vc.hi;
    if (!ok) { FARMS_LIBM_FALLBACK(); sv = sin_dd(x); cv = cos_dd(x); }
    *s = sv;
    *c = cv;
}
__host__ __device__ inline double cr_sin(double x) {
    double s, c;
    cr_sincos(x, &s, &c);
    return s;
}
__host__ __device__ inline double cr_cos(double x) {
    double s, c;
    cr_sincos(x, &s, &c);
    return c;
}
// atan2 for finite nonzero x, y with min/max >= 2^-960 (t and its remainder
// stay normal): atan(t) = atan(c) + atan(u), u = (t - c) / (1 + t c), |u| <=
// 2^-7 + 2^-50, u to ~2^-100 (two quotient digits); atan(u) = u (1 + w), w =
// -u^2/3 in double-double plus the terms u^4..u^8 in double (< 2^-30: rounding
// below 2^-80; truncation u^10 / 11 < 2^-73), atan(c) from the table.
__host__ __device__ inline double cr_atan2(double y, double x) {
    const double ax = __builtin_fabs(x), ay = __builtin_fabs(y);
    const bool swap = ay > ax;
    const double n = swap ? ax : ay, d = swap ? ay : ax;
    // NaN, zero, infinite or badly scaled operands: the full evaluation
    if (!(n > 0.0) || !(d < __builtin_inf()) || !(n >= 0x1p-960 * d)) return atan2_dd(y, x);
    const double qh = n / d;
    const dd t = fast_two_sum(qh, __builtin_fma(-qh, d, n) / d);
    const int j = (int)__builtin_rint(t.hi * 64.0);
    const double cj = (double)j * 0.015625;
    const dd num = fast_two_sum(t.hi - cj, t.lo);          // t.hi - cj exact (Sterbenz; cj = 0 trivially)
    const dd den = dd_add_d(dd_mul_d(t, cj), 1.0);         // 1 + t c
    const double q1 = num.hi / den.hi;
    const dd rem = dd_add(num, dd_neg(dd_mul_d(den, q1)));
    const dd u = fast_two_sum(q1, rem.hi / den.hi);
    dd z = two_prod(u.hi, u.hi);
    z.lo += 2.0 * u.hi * u.lo;
    double tail = __builtin_fma(z.hi, kAtanC[4][0], kAtanC[3][0]);
    tail = __builtin_fma(z.hi, tail, kAtanC[2][0]);
    tail *= z.hi * z.hi;
    const dd w = dd_add_d(dd_mul(z, dd_c(kAtanC[1])), tail);
    const dd au = dd_add(u, dd_mul(u, w));
    dd a = dd_add(dd_c(kAtanTab[j]), au);
    if (swap) a = dd_add(dd{kPio2_hi, kPio2_lo}, dd_neg(a));
    if (__builtin_signbit(x)) a = dd_add(dd{kPi_hi, kPi_lo}, dd_neg(a));
    if (!round_ok(a)) { FARMS_LIBM_FALLBACK(); return atan2_dd(y, x); }
    return __builtin_copysign(a.hi, y);
}

}  // namespace farms_libm

#endif
