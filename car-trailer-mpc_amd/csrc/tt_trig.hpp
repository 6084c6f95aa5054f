// FP64 sin / cos for the kernels' angle arguments: the device library's own algorithm (ROCm 7.2 ocml
// __ocml_sincos_f64 = __ocmlpriv_trigredsmall_f64 + __ocmlpriv_sincosred2_f64 for |x| < 2^30), restated operation by
// operation so that it is bitwise the library's result on that range, but without the library's branch between its
// small- and large-argument reductions.  Straight-line code lets the compiler interleave a stage's independent
// sin / cos evaluations (two or three ~430-cycle dependent chains) instead of running them one after the other.
// The callers take this path only when every lane's arguments are finite and below 2^30 in magnitude (wave-uniform
// test); otherwise they call the library.
#pragma once
#include <hip/hip_runtime.h>

namespace ttmpc {

__device__ __forceinline__ double tt_bits(unsigned long long b) { return __longlong_as_double((long long)b); }

// sin and cos of x, |x| < 2^30 and finite
__device__ __forceinline__ void sincos_small(double x, double& s_out, double& c_out) {
#pragma clang fp contract(off)
    const double ax = fabs(x);
    // argument reduction: ax = t pi/2 + (hi + lo), three-part pi/2 (Cody-Waite with exact products)
    const double t = __builtin_rint(ax * tt_bits(0x3FE45F306DC9C883ull));
    const double r1 = __builtin_fma(t, tt_bits(0xBFF921FB54442D18ull), ax);
    const double r2 = __builtin_fma(t, tt_bits(0xBC91A62633145C00ull), r1);
    const double p = t * tt_bits(0x3C91A62633145C00ull);
    const double pe = __builtin_fma(t, tt_bits(0x3C91A62633145C00ull), -p);
    const double d1 = r1 - p;
    const double d2 = (r1 - d1) - p;
    const double d3 = ((d1 - r2) + d2) - pe;
    const double d4 = __builtin_fma(t, tt_bits(0xB97B839A252049C0ull), d3);
    const double hi = r2 + d4;
    const double lo = d4 - (hi - r2);
    const int q = (int)t & 3;
    // sin and cos of hi + lo on [-pi/4, pi/4]
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
    const double cv = w + __builtin_fma(x4, pc, __builtin_fma(hi, -lo, wc));
    double ps = __builtin_fma(x2, tt_bits(0x3DE5E0B2F9A43BB8ull), tt_bits(0xBE5AE600B42FDFA7ull));
    ps = __builtin_fma(x2, ps, tt_bits(0x3EC71DE3796CDE01ull));
    ps = __builtin_fma(x2, ps, tt_bits(0xBF2A01A019E83E5Cull));
    ps = __builtin_fma(x2, ps, tt_bits(0x3F81111111110BB3ull));
    const double x3 = hi * (-x2);
    const double sa = __builtin_fma(x3, ps, lo * 0.5);
    const double sb = __builtin_fma(x2, sa, -lo);
    const double sv = hi - __builtin_fma(x3, tt_bits(0xBFC5555555555555ull), sb);
    // quadrant: sin = +-(sin | cos), cos = +-(cos | -sin); the sine also takes the sign of x
    const bool even = (q & 1) == 0;
    const unsigned long long neg = q > 1 ? 0x8000000000000000ull : 0ull;
    const unsigned long long sx = (unsigned long long)__double_as_longlong(x) & 0x8000000000000000ull;
    s_out = tt_bits((unsigned long long)__double_as_longlong(even ? sv : cv) ^ sx ^ neg);
    c_out = tt_bits((unsigned long long)__double_as_longlong(even ? cv : -sv) ^ neg);
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
