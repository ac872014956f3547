// akr_trig.h — f64 sin/cos for the path's f32 trig (concentric_disk, GGX sample_wh), host + device.
//
// The reference calls std::sin/std::cos on floats (sampling.h:44-53, microfacet.h:125-149); both
// the oracle and the device evaluate them in f64 and round to f32, which is the
// correctly rounded f32 value except when the f64 result lies within its own error of an f32
// rounding boundary (~2^-29 of inputs).  This is the classic fdlibm construction (Cody-Waite
// reduction by pi/2 in up to three rounds, __kernel_sin / __kernel_cos minimax polynomials, < 1 ulp
// in f64), specialised to |x| < 2^19 pi/2 — the path's arguments are within [-pi, 2 pi].  Larger
// arguments take the general library routine.  It replaces ocml's general sin/cos on the device,
// whose large-argument machinery cost registers and ~4 % of the persistent path kernel.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define AKR_TRIG_HD __host__ __device__ __forceinline__
#else
#define AKR_TRIG_HD inline
#endif

namespace akr {

AKR_TRIG_HD uint32_t trig_hi(double x) {
    uint64_t b;
    memcpy(&b, &x, 8);
    return (uint32_t)(b >> 32);
}
AKR_TRIG_HD double trig_from_hi(uint32_t hi) {  // the double with high word hi and low word 0
    const uint64_t b = (uint64_t)hi << 32;
    double x;
    memcpy(&x, &b, 8);
    return x;
}

// __kernel_sin(x, y, iy): sin(x + y) for |x| <= pi/4, y the tail of the reduced argument
AKR_TRIG_HD double trig_ksin(double x, double y, int iy) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    if ((trig_hi(x) & 0x7fffffffu) < 0x3e400000u && (int)x == 0) return x;  // |x| < 2^-27 (keeps -0)
    const double z = x * x;
    const double v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}

// __kernel_cos(x, y): cos(x + y) for |x| <= pi/4
AKR_TRIG_HD double trig_kcos(double x, double y) {
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const uint32_t ix = trig_hi(x) & 0x7fffffffu;
    if (ix < 0x3e400000u && (int)x == 0) return 1.0;  // |x| < 2^-27
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333u) return 1.0 - (0.5 * z - (z * r - x * y));  // |x| < 0.3
    const double qx = ix > 0x3fe90000u ? 0.28125 : trig_from_hi(ix - 0x00200000u);  // x / 4 (truncated)
    const double hz = 0.5 * z - qx;
    const double a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}

// __ieee754_rem_pio2, medium range (|x| < 2^19 pi/2): x = n pi/2 + y0 + y1
AKR_TRIG_HD int trig_rem_pio2(double x, double &y0, double &y1) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00, pio2_1t = 6.07710050650619224932e-11;
    const double pio2_2 = 6.07710050630396597660e-11, pio2_2t = 2.02226624879595063154e-21;
    const double pio2_3 = 2.02226624871116645580e-21, pio2_3t = 8.47842766036889956997e-32;
    const uint32_t hx = trig_hi(x), ix = hx & 0x7fffffffu;
    const double t = fabs(x);
    const int n = (int)(t * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t - fn * pio2_1;
    double w = fn * pio2_1t;  // first round: good to 85 bits
    const int j = (int)(ix >> 20);
    y0 = r - w;
    int i = j - (int)((trig_hi(y0) >> 20) & 0x7ff);
    if (i > 16) {  // second round: good to 118 bits
        double tt = r;
        w = fn * pio2_2;
        r = tt - w;
        w = fn * pio2_2t - ((tt - r) - w);
        y0 = r - w;
        i = j - (int)((trig_hi(y0) >> 20) & 0x7ff);
        if (i > 49) {  // third round: 151 bits
            tt = r;
            w = fn * pio2_3;
            r = tt - w;
            w = fn * pio2_3t - ((tt - r) - w);
            y0 = r - w;
        }
    }
    y1 = (r - y0) - w;
    if ((int32_t)hx < 0) {
        y0 = -y0;
        y1 = -y1;
        return -n;
    }
    return n;
}

// sin / cos of an f32 argument, evaluated in f64 and rounded to f32
AKR_TRIG_HD float trig_sinf(float xf) {
    const double x = (double)xf;
    const uint32_t ix = trig_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return (float)trig_ksin(x, 0.0, 0);  // |x| <= pi/4
    if (ix >= 0x413921fbu) return (float)sin(x);                // |x| >= 2^19 pi/2, inf, NaN
    double y0, y1;
    const int n = trig_rem_pio2(x, y0, y1);
    double s;
    switch (n & 3) {
        case 0: s = trig_ksin(y0, y1, 1); break;
        case 1: s = trig_kcos(y0, y1); break;
        case 2: s = -trig_ksin(y0, y1, 1); break;
        default: s = -trig_kcos(y0, y1); break;
    }
    return (float)s;
}

AKR_TRIG_HD float trig_cosf(float xf) {
    const double x = (double)xf;
    const uint32_t ix = trig_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) return (float)trig_kcos(x, 0.0);
    if (ix >= 0x413921fbu) return (float)cos(x);
    double y0, y1;
    const int n = trig_rem_pio2(x, y0, y1);
    double c;
    switch (n & 3) {
        case 0: c = trig_kcos(y0, y1); break;
        case 1: c = -trig_ksin(y0, y1, 1); break;
        case 2: c = -trig_kcos(y0, y1); break;
        default: c = trig_ksin(y0, y1, 1); break;
    }
    return (float)c;
}

// sin and cos of one f32 argument with one reduction: the same values as trig_sinf / trig_cosf.
// On the device |x| >= 2^19 pi/2 (and inf / NaN) gives NaN instead of the library call: the path's
// arguments are 2 pi u and pi/4 ratios of sampler draws u in [0, 1] (sampling.h:44-53,
// microfacet.h:130), so that branch is unreachable there and a call would cost registers.
AKR_TRIG_HD void trig_sincosf(float xf, float &sf, float &cf) {
    const double x = (double)xf;
    const uint32_t ix = trig_hi(x) & 0x7fffffffu;
    if (ix <= 0x3fe921fbu) {
        sf = (float)trig_ksin(x, 0.0, 0);
        cf = (float)trig_kcos(x, 0.0);
        return;
    }
    if (ix >= 0x413921fbu) {
#if defined(__HIP_DEVICE_COMPILE__)
        sf = cf = __builtin_nanf("");
#else
        sf = (float)sin(x);
        cf = (float)cos(x);
#endif
        return;
    }
    double y0, y1;
    const int n = trig_rem_pio2(x, y0, y1);
    const double ks = trig_ksin(y0, y1, 1), kc = trig_kcos(y0, y1);
    switch (n & 3) {
        case 0: sf = (float)ks; cf = (float)kc; break;
        case 1: sf = (float)kc; cf = (float)-ks; break;
        case 2: sf = (float)-ks; cf = (float)-kc; break;
        default: sf = (float)-kc; cf = (float)ks; break;
    }
}

}  // namespace akr
