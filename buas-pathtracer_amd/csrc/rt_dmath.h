// rt_dmath.h — device math for the gfx950 path tracer.
//
// Reproduces MathLib semantics (MathLib/my_math.h) operation for operation:
// V3 ops component-wise, dot = (ax*bx + ay*by) + az*bz, min/max as the
// reference's ternaries (NaN behaviour included), noz / transform /
// transform_normal with the reference's quirks.  Transcendentals follow the
// deterministic Cephes single-precision spec that the CPU oracle restates
// (DESIGN.md §Numerics).  Built with -ffp-contract=off and correctly rounded
// division / sqrt so results are bit-comparable with the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/rt_abi.h"

#ifdef RT_DMATH_HOST_TEST        // tools/check_sincos.cpp: the device math compiled for the host
#define RT_D inline
#else
#define RT_D __device__ __forceinline__
#endif

namespace rtd {

constexpr float PI_32 = 3.14159265359f;    // MathLib/my_math.h:15
constexpr float TAU_32 = 6.28318530717f;   // :16
constexpr float EPSILON = 0.001f;          // RT/common.h:35
constexpr float FLT_MAX_ = 3.402823466e+38F;

struct V3 { float x, y, z; };
struct V2 { float x, y; };

RT_D V3 v3(float x, float y, float z) { return {x, y, z}; }
RT_D V3 v3s(float s) { return {s, s, s}; }
RT_D V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_D V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_D V3 mul(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_D V3 divv(V3 a, V3 b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
RT_D V3 muls(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
RT_D V3 smul(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
RT_D V3 divs(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
RT_D V3 sdiv(float s, V3 a) { return {s / a.x, s / a.y, s / a.z}; }
RT_D V3 neg(V3 a) { return {-a.x, -a.y, -a.z}; }
// 1.0f / x, correctly rounded, in 3 VALU instead of the 11-instruction division
// expansion (div_scale x2, rcp, 5 fma, mul, div_fmas, div_fixup): v_rcp_f32's estimate
// refined by one Newton step on the FMA residual, for |x| in [2^-125, 2^125], where
// neither the residual nor the result leaves the normal range.  Other inputs (zeros,
// denormals, huge values, inf, NaN) take the full division; a wave whose lanes are all
// in range skips it.  rt_debug_verify_rcp checks it against the IEEE division for
// every one of the 2^32 floats (tests/test_gpu_parity.py::test_rcp_cr_exhaustive).  The host
// build of tools/check_sincos.cpp has no v_rcp_f32 and divides (the same bits).
RT_D float rcp_cr(float x) {
#ifndef RT_DMATH_HOST_TEST
    const float a = __builtin_fabsf(x);
    if (a >= 0x1p-125f && a <= 0x1p125f) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
#endif
    return 1.0f / x;
}
RT_D V3 rcp3(V3 a) { return {rcp_cr(a.x), rcp_cr(a.y), rcp_cr(a.z)}; }
RT_D float dot(V3 a, V3 b) { return a.x*b.x + a.y*b.y + a.z*b.z; }
RT_D V3 cross(V3 a, V3 b) { return {a.y*b.z - a.z*b.y, a.z*b.x - a.x*b.z, a.x*b.y - a.y*b.x}; }
RT_D float length_sq(V3 a) { return dot(a, a); }
RT_D float mn(float a, float b) { return a < b ? a : b; }
RT_D float mx(float a, float b) { return a > b ? a : b; }
RT_D float clampf_(float n, float a, float b) { return mx(a, mn(b, n)); }
RT_D float max3(V3 a) { return mx(a.x, mx(a.y, a.z)); }
RT_D V3 vabs(V3 a) { return {fabsf(a.x), fabsf(a.y), fabsf(a.z)}; }
RT_D V3 normalize(V3 a) { float r = rcp_cr(__builtin_sqrtf(dot(a, a))); return muls(a, r); }
RT_D V3 noz(V3 a) {
    V3 r = {0.0f, 0.0f, 0.0f};
    float lsq = length_sq(a);
    if ((lsq > 0.0001f) && (lsq < __builtin_inff())) r = divs(a, __builtin_sqrtf(lsq));
    return r;
}
RT_D float lerpf_(float a, float b, float t) { return a*(1.0f - t) + b*t; }
RT_D V3 lerp3(V3 a, V3 b, float t) { return add(muls(a, 1.0f - t), muls(b, t)); }
RT_D V3 reflect(V3 v, V3 n) { return sub(v, muls(n, 2.0f*dot(v, n))); }
RT_D float sign_of(float x) { return x < 0.0f ? -1.0f : 1.0f; }
RT_D float copy_sign(float v, float s) {
    return __uint_as_float((__float_as_uint(s) & 0x80000000u) | (__float_as_uint(v) & 0x7FFFFFFFu));
}
RT_D float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// 3x4 affine rows of an M4x4 (the 4th row is never read by transform()).
struct M34 { float e[3][4]; };

RT_D V3 xform(const M34& a, V3 p, float pw) {               // MathLib/my_math.h:947-954
    return {p.x*a.e[0][0] + p.y*a.e[0][1] + p.z*a.e[0][2] + pw*a.e[0][3],
            p.x*a.e[1][0] + p.y*a.e[1][1] + p.z*a.e[1][2] + pw*a.e[1][3],
            p.x*a.e[2][0] + p.y*a.e[2][1] + p.z*a.e[2][2] + pw*a.e[2][3]};
}
RT_D V3 xform_normal(const M34& a, V3 n) {                  // :956-963 (quirk kept)
    return {n.x*a.e[0][0] + n.y*a.e[0][1] + n.z*a.e[2][0],
            n.x*a.e[0][1] + n.y*a.e[1][1] + n.z*a.e[2][1],
            n.x*a.e[0][2] + n.y*a.e[1][2] + n.z*a.e[2][2]};
}

// ---- deterministic transcendentals (Cephes single precision; same spec as oracle)
RT_D float sin_poly(float x, float z) {
    return ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
}
RT_D float cos_poly(float z) {
    return ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z
           - 0.5f * z + 1.0f;
}
constexpr float FOPI = 1.27323954473516f;
constexpr float DP1 = 0.78515625f;
constexpr float DP2 = 2.4187564849853515625e-4f;
constexpr float DP3 = 3.77489497744594108e-8f;

RT_D float d_sinf(float xx) {
    float x = xx;
    int sgn = 0;
    if (x < 0.0f) { sgn = 1; x = -x; }
    if (!(x < 8192.0f)) return (x == x) ? 0.0f : x;
    uint32_t j = (uint32_t)(FOPI * x);
    float y = (float)j;
    if (j & 1u) { j += 1u; y += 1.0f; }
    j &= 7u;
    if (j > 3u) { sgn ^= 1; j -= 4u; }
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float r = (j == 1u || j == 2u) ? cos_poly(z) : sin_poly(x, z);
    return sgn ? -r : r;
}
RT_D float d_cosf(float xx) {
    float x = fabsf(xx);
    if (!(x < 8192.0f)) return (x == x) ? 1.0f : x;
    uint32_t j = (uint32_t)(FOPI * x);
    float y = (float)j;
    if (j & 1u) { j += 1u; y += 1.0f; }
    j &= 7u;
    int sgn = 0;
    if (j > 3u) { j -= 4u; sgn ^= 1; }
    if (j > 1u) sgn ^= 1;
    x = ((x - y * DP1) - y * DP2) - y * DP3;
    float z = x * x;
    float r = (j == 1u || j == 2u) ? sin_poly(x, z) : cos_poly(z);
    return sgn ? -r : r;
}
// sin and cos of one argument (map_to_hemisphere, the bokeh sample): one range reduction and one
// evaluation of each polynomial for both, the same operations as d_sinf / d_cosf, so the same bits
// (a -0 argument reduces to +0 here, where d_sinf keeps -0; both give sin(-0) = +0 through sin_poly)
RT_D void d_sincosf(float xx, float& s_out, float& c_out) {
    const float x0 = fabsf(xx);
    if (!(x0 < 8192.0f)) {
        s_out = (xx == xx) ? 0.0f : xx;
        c_out = (x0 == x0) ? 1.0f : x0;
        return;
    }
    uint32_t j = (uint32_t)(FOPI * x0);
    float y = (float)j;
    if (j & 1u) { j += 1u; y += 1.0f; }
    j &= 7u;
    int ss = xx < 0.0f ? 1 : 0, cs = 0;
    if (j > 3u) { j -= 4u; ss ^= 1; cs ^= 1; }
    if (j > 1u) cs ^= 1;
    const float x = ((x0 - y * DP1) - y * DP2) - y * DP3;
    const float z = x * x;
    const float sp = sin_poly(x, z), cp = cos_poly(z);
    const bool swap = j == 1u || j == 2u;
    const float rs = swap ? cp : sp, rc = swap ? sp : cp;
    s_out = ss ? -rs : rs;
    c_out = cs ? -rc : rc;
}
RT_D float d_ldexp(float y, int n) {
    if (n > 127) { y = y * __uint_as_float(0x7F000000u); n -= 127; if (n > 127) n = 127; }
    if (n < -126) { y = y * __uint_as_float(0x00800000u); n += 126; if (n < -126) n = -126; }
    return y * __uint_as_float((uint32_t)(n + 127) << 23);
}
RT_D float d_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283905206835f) return __builtin_inff();
    if (x < -103.278929903431851103f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    z = x * x;
    float y = ((((( 1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x
                 + 4.1665795894E-2f) * x + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    return d_ldexp(y, n);
}
RT_D float d_logf(float x) {
    if (x != x) return x;
    if (x <= 0.0f) return x == 0.0f ? -__builtin_inff() : __builtin_nanf("");
    if (x == __builtin_inff()) return x;
    uint32_t u = __float_as_uint(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 16777216.0f; e = -24; u = __float_as_uint(x); }
    e += (int)((u >> 23) & 0xFFu) - 126;
    x = __uint_as_float((u & 0x807FFFFFu) | 0x3F000000u);
    if (x < 0.707106781186547524f) { e -= 1; x = x + x - 1.0f; }
    else { x = x - 1.0f; }
    float z = x * x;
    float y = (((((((( 7.0376836292E-2f * x - 1.1514610310E-1f) * x + 1.1676998740E-1f) * x
                  - 1.2420140846E-1f) * x + 1.4249322787E-1f) * x - 1.6668057665E-1f) * x
                  + 2.0000714765E-1f) * x - 2.4999993993E-1f) * x + 3.3333331174E-1f) * x * z;
    float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    z = x + y;
    z = z + 0.693359375f * fe;
    return z;
}
RT_D float d_powf(float x, float y) { return d_expf(y * d_logf(x)); }
RT_D float d_atanf(float xx) {
    float x = xx;
    int sgn = 0;
    if (x < 0.0f) { sgn = 1; x = -x; }
    float y;
    if (x > 2.414213562373095f) { y = 1.5707963267948966192f; x = -rcp_cr(x); }
    else if (x > 0.4142135623730950f) { y = 0.7853981633974483096f; x = (x - 1.0f) / (x + 1.0f); }
    else { y = 0.0f; }
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z
              - 3.33329491539E-1f) * z * x + x);
    return sgn ? -y : y;
}
RT_D float d_atan2f(float y, float x) {
    if (x != x || y != y) return x + y;
    if (x == 0.0f) {
        if (y > 0.0f) return 1.5707963267948966192f;
        if (y < 0.0f) return -1.5707963267948966192f;
        return 0.0f;
    }
    if (y == 0.0f) return (x > 0.0f) ? 0.0f : 3.14159265358979323846f;
    float w;
    if (x < 0.0f) w = (y < 0.0f) ? -3.14159265358979323846f : 3.14159265358979323846f;
    else w = 0.0f;
    return w + d_atanf(y / x);
}
RT_D float d_asinf(float xx) {
    float a = fabsf(xx);
    if (a > 1.0f) return __builtin_nanf("");
    if (a < 1.0e-4f) return xx;
    float x, z;
    int flag;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); x = __builtin_sqrtf(z); flag = 1; }
    else { x = a; z = x * x; flag = 0; }
    z = (((( 4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z
          + 7.4953002686E-2f) * z + 1.6666752422E-1f) * z * x + x;
    if (flag) { z = z + z; z = 1.5707963267948966192f - z; }
    return xx < 0.0f ? -z : z;
}

// ---- RNG (RT/samplers.h:3-108)
RT_D uint32_t wang_hash(uint32_t key) {
    key += ~(key << 15);
    key ^= (key >> 10);
    key += (key << 3);
    key ^= (key >> 6);
    key += ~(key << 11);
    key ^= (key >> 16);
    return key;
}
RT_D uint32_t hash_coordinate3(uint32_t x, uint32_t y, uint32_t z) {
    return (x*73856093u) ^ (y*83492791u) ^ (z*871603259u);
}
RT_D uint32_t hash_coordinate2(uint32_t x, uint32_t y) {
    uint32_t qx = 1103515245u*((x >> 1) ^ y);
    uint32_t qy = 1103515245u*((y >> 1) ^ x);
    return 1103515245u*(qx ^ (qy >> 3));
}

struct Rng { uint32_t e0, e1, e2, e3; };   // RandomSeries: 4 xorshift32 lanes

RT_D uint32_t xs(uint32_t r) { r ^= r << 13; r ^= r >> 17; r ^= r << 5; return r; }
RT_D void next_set(Rng& s) { s.e0 = xs(s.e0); s.e1 = xs(s.e1); s.e2 = xs(s.e2); s.e3 = xs(s.e3); }
RT_D float unit_from_bits(uint32_t b) { return __uint_as_float((127u << 23) | (b >> 9)) - 1.0f; }
// random_unilaterals(): advances all four lanes, returns them as floats in [0,1)
RT_D void unilaterals(Rng& s, float& a, float& b, float& c, float& d) {
    next_set(s);
    a = unit_from_bits(s.e0); b = unit_from_bits(s.e1); c = unit_from_bits(s.e2); d = unit_from_bits(s.e3);
}
RT_D Rng random_seed(uint32_t seed) {                        // RT/samplers.h:92-108
    if (seed == 0) seed = 0xFFFFFFFFu;
    uint32_t h = wang_hash(seed);
    Rng r = {h, h, h, h};
    next_set(r); uint32_t a0 = r.e0;
    next_set(r); uint32_t b1 = r.e1;
    next_set(r); uint32_t c2 = r.e2;
    next_set(r);
    r.e0 = wang_hash(a0); r.e1 = wang_hash(b1); r.e2 = wang_hash(c2);
    return r;
}
// per-sample seed: tile seed of RT/raytracer.cpp:588-590 keyed by pixel and sample
RT_D uint32_t sample_seed(uint32_t total_frame_index, uint32_t frame_count, uint32_t tile_index,
                          uint32_t pixel_id, uint32_t canonical) {
    uint32_t tile_seed = hash_coordinate3(total_frame_index, frame_count, tile_index);
    return wang_hash(tile_seed ^ wang_hash((pixel_id * 0x9E3779B9u) ^ wang_hash(canonical + 0x68E31DA4u)));
}

}  // namespace rtd
