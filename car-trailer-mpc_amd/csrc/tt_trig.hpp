// FP64 sin / cos for the kernels' angle arguments: the device library's own algorithm (ROCm 7.2 ocml
// __ocml_sincos_f64 = __ocmlpriv_trigredsmall_f64 + __ocmlpriv_sincosred2_f64 for |x| < 2^30), restated operation by
// operation so that it is bitwise the library's result on that range, but without the library's branch between its
// small- and large-argument reductions.  Straight-line code lets the compiler interleave a stage's independent
// sin / cos evaluations (two or three ~430-cycle dependent chains) instead of running them one after the other.
// The callers take this path only when every lane's arguments are finite and below 2^30 in magnitude (wave-uniform
// test); otherwise they call the library.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_version.h>

// The restatement is checked bit for bit against THIS ROCm's ocml (tools/trig_check.hip, run by
// tests/test_gpu_trig.py on every GPU test session).  Another ROCm may change ocml's constants or operation order, and
// the kernels would drift silently from the library and from the lockstep parity the OBCA tests rely on: refuse to
// build until trig_check has been re-run there (then extend this test, or build with -DTT_TRIG_UNCHECKED_ROCM).
#if !(HIP_VERSION_MAJOR == 7 && HIP_VERSION_MINOR == 2) && !defined(TT_TRIG_UNCHECKED_ROCM)
#error "tt_trig.hpp restates ROCm 7.2's ocml sin/cos/tan: re-run tools/trig_check on this ROCm before building"
#endif

namespace ttmpc {

__device__ __forceinline__ double tt_bits(unsigned long long b) { return __longlong_as_double((long long)b); }

// argument reduction of ax = |x| < 2^30: ax = t pi/2 + (hi + lo), three-part pi/2 (Cody-Waite with exact products);
// q = t mod 4 (ocml __ocmlpriv_trigredsmall_f64)
__device__ __forceinline__ void trigred_small(double ax, double& hi, double& lo, int& q) {
#pragma clang fp contract(off)
    const double t = __builtin_rint(ax * tt_bits(0x3FE45F306DC9C883ull));
    const double r1 = __builtin_fma(t, tt_bits(0xBFF921FB54442D18ull), ax);
    const double r2 = __builtin_fma(t, tt_bits(0xBC91A62633145C00ull), r1);
    const double p = t * tt_bits(0x3C91A62633145C00ull);
    const double pe = __builtin_fma(t, tt_bits(0x3C91A62633145C00ull), -p);
    const double d1 = r1 - p;
    const double d2 = (r1 - d1) - p;
    const double d3 = ((d1 - r2) + d2) - pe;
    const double d4 = __builtin_fma(t, tt_bits(0xB97B839A252049C0ull), d3);
    hi = r2 + d4;
    lo = d4 - (hi - r2);
    q = (int)t & 3;
}
// sin and cos of hi + lo on [-pi/4, pi/4] (ocml __ocmlpriv_sincosred2_f64)
__device__ __forceinline__ void sincosred2(double hi, double lo, double& sv, double& cv) {
#pragma clang fp contract(off)
    const double x2 = hi * hi;
    const double h = x2 * 0.5;
    const double w = 1.0 - h;
    const double wc = (1.0 - w) - h;
    const double x4 = x2 * x2;
    double pc = __builtin_fma(x2, tt_bits(0xBDA907DB46CC5E42ull), tt_bits(0x3E21EEB69037AB78ull));
    pc = __builtin_fma(x2, pc, tt_bits(0xBE927E4FA17F65F6ull));
    pc = __builtin_fma(x2, pc, tt_bits(0x3EFA01A019F4EC90ull));
    pc = __builtin_fma(x2, pc, tt_bits(0xBF56C16C16C16967ull));
    pc = __builtin_fma(x2, pc, tt_bits(0x3FA5555555555555ull));
    cv = w + __builtin_fma(x4, pc, __builtin_fma(hi, -lo, wc));
    double ps = __builtin_fma(x2, tt_bits(0x3DE5E0B2F9A43BB8ull), tt_bits(0xBE5AE600B42FDFA7ull));
    ps = __builtin_fma(x2, ps, tt_bits(0x3EC71DE3796CDE01ull));
    ps = __builtin_fma(x2, ps, tt_bits(0xBF2A01A019E83E5Cull));
    ps = __builtin_fma(x2, ps, tt_bits(0x3F81111111110BB3ull));
    const double x3 = hi * (-x2);
    const double sa = __builtin_fma(x3, ps, lo * 0.5);
    const double sb = __builtin_fma(x2, sa, -lo);
    sv = hi - __builtin_fma(x3, tt_bits(0xBFC5555555555555ull), sb);
}
// tan of hi + lo on [-pi/4, pi/4], or -1/tan when odd (ocml __ocmlpriv_tanred2_f64)
__device__ __forceinline__ double tanred2(double x, double y, bool odd) {
#pragma clang fp contract(off)
    const double x2 = x * x;
    const double s = x2 + __builtin_fma(x, y * 2.0, __builtin_fma(x, x, -x2));
    double p = __builtin_fma(s, tt_bits(0x3EF5E089C751C08Cull), tt_bits(0xBF078809A9A29F71ull));
    p = __builtin_fma(s, p, tt_bits(0x3F17746F90A8AAE0ull));
    p = __builtin_fma(s, p, tt_bits(0xBEFBB44DA6FBF144ull));
    p = __builtin_fma(s, p, tt_bits(0x3F21E634A7943ACFull));
    p = __builtin_fma(s, p, tt_bits(0x3F2D250FDEB68FEBull));
    p = __builtin_fma(s, p, tt_bits(0x3F437FD9B58C4D95ull));
    p = __builtin_fma(s, p, tt_bits(0x3F57D5AF15120E2Cull));
    p = __builtin_fma(s, p, tt_bits(0x3F6D6D93E09491DFull));
    p = __builtin_fma(s, p, tt_bits(0x3F8226E12033784Dull));
    p = __builtin_fma(s, p, tt_bits(0x3F9664F49AC36AE2ull));
    p = __builtin_fma(s, p, tt_bits(0x3FABA1BA1B451C21ull));
    p = __builtin_fma(s, p, tt_bits(0x3FC11111111185B7ull));
    p = __builtin_fma(s, p, tt_bits(0x3FD55555555554EEull));
    const double sp = s * p;
    const double a = x * sp;
    const double ae = __builtin_fma(x, sp, -a);
    const double b = x + a;
    const double be = a - (b - x);
    const double cc = (y + ae) + be;
    const double th = b + cc;
    const double tl = cc - (th - b);
    const double r0 = __builtin_amdgcn_rcp(th);
    const double r1 = __builtin_fma(__builtin_fma(-th, r0, 1.0), r0, r0);
    const double r = __builtin_fma(__builtin_fma(-th, r1, 1.0), r1, r1);
    const double m = th * r;
    const double e = __builtin_fma(r, tl, __builtin_fma(r, th, -m));
    const double u = m + e;
    const double ue = e - (u - m);
    const double v = 1.0 - u;
    const double ve = (((1.0 - v) - u) - ue);
    const double it = r + r * (v + ve);
    return odd ? -it : th;
}
__device__ __forceinline__ unsigned long long tt_u(double v) { return (unsigned long long)__double_as_longlong(v); }
constexpr unsigned long long kSign = 0x8000000000000000ull;

// sin and cos of x, |x| < 2^30 and finite (ocml __ocml_sincos_f64)
__device__ __forceinline__ void sincos_small(double x, double& s_out, double& c_out) {
    double hi, lo, sv, cv;
    int q;
    trigred_small(fabs(x), hi, lo, q);
    sincosred2(hi, lo, sv, cv);
    // quadrant: sin = +-(sin | cos), cos = +-(cos | -sin); the sine also takes the sign of x
    const bool even = (q & 1) == 0;
    const unsigned long long neg = q > 1 ? kSign : 0ull;
    s_out = tt_bits(tt_u(even ? sv : cv) ^ (tt_u(x) & kSign) ^ neg);
    c_out = tt_bits(tt_u(even ? cv : -sv) ^ neg);
}
// tan and cos of x, |x| < 2^30 and finite, one reduction for both (ocml __ocml_tan_f64, __ocml_cos_f64)
__device__ __forceinline__ void tancos_small(double x, double& t_out, double& c_out) {
    double hi, lo, sv, cv;
    int q;
    trigred_small(fabs(x), hi, lo, q);
    sincosred2(hi, lo, sv, cv);
    const bool even = (q & 1) == 0;
    c_out = tt_bits(tt_u(even ? cv : -sv) ^ (q > 1 ? kSign : 0ull));
    t_out = tt_bits(tt_u(tanred2(hi, lo, !even)) ^ (tt_u(x) & kSign));
}

// true when the fast path is exact for every lane of the wave (wave-uniform)
__device__ __forceinline__ bool sincos_small_ok(bool lane_ok) { return __builtin_amdgcn_ballot_w64(!lane_ok) == 0ull; }
__device__ __forceinline__ bool sincos_arg_ok(double x) { return fabs(x) < 1073741824.0; }  // 2^30; false for NaN / inf

// independent sin / cos pairs of a stage: the straight-line path when every active lane's arguments qualify, else the library
__device__ __forceinline__ void sincos2(double a, double& sa, double& ca, double b, double& sb, double& cb) {
    if (sincos_small_ok(sincos_arg_ok(a) && sincos_arg_ok(b))) {
        sincos_small(a, sa, ca);
        sincos_small(b, sb, cb);
    } else {
        sincos(a, &sa, &ca);
        sincos(b, &sb, &cb);
    }
}
// sin / cos of a and b, tan and cos of c (the OBCA model's theta, psi, phi)
__device__ __forceinline__ void sincos2_tancos(double a, double& sa, double& ca, double b, double& sb, double& cb, double c,
                                               double& tc, double& cc) {
    if (sincos_small_ok(sincos_arg_ok(a) && sincos_arg_ok(b) && sincos_arg_ok(c))) {
        sincos_small(a, sa, ca);
        sincos_small(b, sb, cb);
        tancos_small(c, tc, cc);
    } else {
        sincos(a, &sa, &ca);
        sincos(b, &sb, &cb);
        tc = tan(c);
        cc = cos(c);
    }
}
__device__ __forceinline__ void sincos3(double a, double& sa, double& ca, double b, double& sb, double& cb, double c,
                                        double& sc, double& cc) {
    if (sincos_small_ok(sincos_arg_ok(a) && sincos_arg_ok(b) && sincos_arg_ok(c))) {
        sincos_small(a, sa, ca);
        sincos_small(b, sb, cb);
        sincos_small(c, sc, cc);
    } else {
        sincos(a, &sa, &ca);
        sincos(b, &sb, &cb);
        sincos(c, &sc, &cc);
    }
}

}  // namespace ttmpc
