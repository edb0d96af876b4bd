/*
 * libm_f32.h — fp32 atan2f with the exact operation sequence of the Sun fdlibm algorithm that
 * glibc's generic flt-32 libm uses (e_atan2f.c / s_atanf.c). The reference computes the azimuth
 * with std::atan2(float,float) = atan2f (src/scanRegistration.cpp:56,141,208); ocml's atan2f
 * differs from glibc's in the last ulp for ~16% of inputs, which would change the bits of every
 * point's `intensity` (= scanID + 0.1*relTime). This restatement is pinned bit-exact against the
 * host glibc atan2f by tests/test_libm_pin.py (same source compiled for the host).
 *
 * Compile with -ffp-contract=off: every operation below must round separately.
 * Usable from host and device code.
 */
#ifndef ALOAM_LIBM_F32_H
#define ALOAM_LIBM_F32_H
#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define LIBM_FN __host__ __device__ static inline
#else
#define LIBM_FN static inline
#endif

LIBM_FN int32_t lm_f2i(float f) { int32_t i; memcpy(&i, &f, 4); return i; }
LIBM_FN float lm_fabsf(float x) { int32_t i = lm_f2i(x) & 0x7fffffff; float r; memcpy(&r, &i, 4); return r; }

LIBM_FN float lm_atanf(float x) {
    const float atanhi[4] = {4.6364760399e-01f, 7.8539812565e-01f, 9.8279368877e-01f, 1.5707962513e+00f};
    const float atanlo[4] = {5.0121582440e-09f, 3.7748947079e-08f, 3.4473217170e-08f, 7.5497894159e-08f};
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const float one = 1.0f;
    int32_t hx = lm_f2i(x), ix = hx & 0x7fffffff, id;
    if (ix >= 0x4c000000) {                       /* |x| >= 2^25 */
        if (ix > 0x7f800000) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3ee00000) {                        /* |x| < 0.4375 */
        if (ix < 0x31000000) return x;            /* |x| < 2^-29 */
        id = -1;
    } else {
        x = lm_fabsf(x);
        if (ix < 0x3f980000) {                    /* |x| < 1.1875 */
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - one) / (2.0f + x); }
            else { id = 1; x = (x - one) / (x + one); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (one + 1.5f * x); }
            else { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return (hx < 0) ? -z : z;
}

LIBM_FN float lm_atan2f(float y, float x) {
    const float pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f, tiny = 1.0e-30f;
    int32_t hx = lm_f2i(x), ix = hx & 0x7fffffff, hy = lm_f2i(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;
    if (hx == 0x3f800000) return lm_atanf(y);
    int32_t m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        switch (m) { case 0: case 1: return y; case 2: return pi + tiny; default: return -pi - tiny; }
    }
    if (ix == 0) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        const float pi_o_4 = 7.8539818525e-01f;
        if (iy == 0x7f800000) {
            switch (m) { case 0: return pi_o_4 + tiny; case 1: return -pi_o_4 - tiny;
                         case 2: return 3.0f * pi_o_4 + tiny; default: return -3.0f * pi_o_4 - tiny; }
        } else {
            switch (m) { case 0: return 0.0f; case 1: return -0.0f; case 2: return pi + tiny; default: return -pi - tiny; }
        }
    }
    if (iy == 0x7f800000) return (hy < 0) ? -pi_o_2 - tiny : pi_o_2 + tiny;
    int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;          /* |y/x| > 2^60 (glibc keeps Sun's 60) */
    else if (hx < 0 && k < -60) z = 0.0f;            /* |y|/x > -2^-60 */
    else z = lm_atanf(lm_fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}
#endif
