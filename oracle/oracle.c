/*
 * oracle.c — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE
 * ONLY (see oracle.h): the parity checker and the CPU baseline, never the
 * product.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off, no fast-math).
 *
 * Every function cites the reference file:line it restates.  Expression
 * order follows the reference's MathLib operator definitions
 * (MathLib/my_math.h) so that float rounding matches: V3 ops are evaluated
 * component-wise left to right, dot = (ax*bx + ay*by) + az*bz, etc.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <stdatomic.h>
#include <time.h>

/* ====================================================================== */
/* Scalars and vectors (MathLib/my_math.h)                                */
/* ====================================================================== */

#define PI_32   3.14159265359f          /* MathLib/my_math.h:15 */
#define TAU_32  6.28318530717f          /* MathLib/my_math.h:16 */
#define EPSILON 0.001f                  /* RT/common.h:35 */

typedef rt_v3 V3;
typedef struct { float x, y; } V2;

static inline float mn(float a, float b) { return a < b ? a : b; }      /* my_math.h:78 */
static inline float mx(float a, float b) { return a > b ? a : b; }      /* my_math.h:83 */
static inline float clampf_(float n, float a, float b) { return mx(a, mn(b, n)); } /* :108 */
static inline float absf(float x) { return fabsf(x); }
static inline float sign_of(float x) { return x < 0.0f ? -1.0f : 1.0f; }  /* :168 */
static inline float copy_sign(float v, float s) {                          /* :186 */
    uint32_t vb, sb; memcpy(&vb, &v, 4); memcpy(&sb, &s, 4);
    vb = (sb & 0x80000000u) | (vb & 0x7FFFFFFFu);
    float r; memcpy(&r, &vb, 4); return r;
}
static inline float lerpf_(float a, float b, float t) { return a*(1.0f - t) + b*t; } /* :70 */

static inline V3 v3(float x, float y, float z) { V3 r = { x, y, z }; return r; }
static inline V3 v3s(float s) { V3 r = { s, s, s }; return r; }
static inline V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline V3 divv(V3 a, V3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline V3 muls(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }   /* V3*float */
static inline V3 smul(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }   /* float*V3 */
static inline V3 divs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline V3 sdiv(float s, V3 a) { return v3(s / a.x, s / a.y, s / a.z); }
static inline V3 neg(V3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float dot(V3 a, V3 b) { return a.x*b.x + a.y*b.y + a.z*b.z; }      /* :454 */
static inline V3 cross(V3 a, V3 b) {                                              /* :459 */
    return v3(a.y*b.z - a.z*b.y, a.z*b.x - a.x*b.z, a.x*b.y - a.y*b.x);
}
static inline float length_sq(V3 a) { return dot(a, a); }
static inline float length_(V3 a) { return sqrtf(dot(a, a)); }
static inline V3 normalize(V3 a) { float r = 1.0f / length_(a); return muls(a, r); } /* :487 */
static inline V3 noz(V3 a) {                                                      /* :493 */
    V3 r = v3(0, 0, 0);
    float lsq = length_sq(a);
    if ((lsq > 0.0001f) && (lsq < INFINITY)) r = divs(a, sqrtf(lsq));
    return r;
}
static inline V3 lerp3(V3 a, V3 b, float t) { return add(muls(a, 1.0f - t), muls(b, t)); } /* :449 */
static inline V3 reflect(V3 v, V3 n) { return sub(v, muls(n, 2.0f*dot(v, n))); } /* :472 */
static inline V3 vabs(V3 a) { return v3(absf(a.x), absf(a.y), absf(a.z)); }
static inline V3 vmin(V3 a, V3 b) { return v3(mn(a.x, b.x), mn(a.y, b.y), mn(a.z, b.z)); }
static inline V3 vmax(V3 a, V3 b) { return v3(mx(a.x, b.x), mx(a.y, b.y), mx(a.z, b.z)); }
static inline float max3(V3 a) { return mx(a.x, mx(a.y, a.z)); }                 /* :536 */
static inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* transform(m, p, pw) MathLib/my_math.h:947-954 */
static inline V3 xform(const rt_m4x4* a, V3 p, float pw) {
    V3 r;
    r.x = p.x*a->e[0][0] + p.y*a->e[0][1] + p.z*a->e[0][2] + pw*a->e[0][3];
    r.y = p.x*a->e[1][0] + p.y*a->e[1][1] + p.z*a->e[1][2] + pw*a->e[1][3];
    r.z = p.x*a->e[2][0] + p.y*a->e[2][1] + p.z*a->e[2][2] + pw*a->e[2][3];
    return r;
}
/* transform_normal MathLib/my_math.h:956-963 — non-transposed quirk kept (e[0][1] in x). */
static inline V3 xform_normal(const rt_m4x4* a, V3 n) {
    V3 r;
    r.x = n.x*a->e[0][0] + n.y*a->e[0][1] + n.z*a->e[2][0];
    r.y = n.x*a->e[0][1] + n.y*a->e[1][1] + n.z*a->e[2][1];
    r.z = n.x*a->e[0][2] + n.y*a->e[1][2] + n.z*a->e[2][2];
    return r;
}
static inline V3 translation(const rt_m4x4* a) { return v3(a->e[0][3], a->e[1][3], a->e[2][3]); } /* :978 */

/* ====================================================================== */
/* Deterministic transcendentals (spec shared with the HIP kernels).       */
/* Cephes single-precision algorithms (S. L. Moshier), restated.           */
/* ====================================================================== */

static inline float bits_f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f_bits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float sin_poly(float x, float z) {
    return ((-1.9515295891E-4f * z + 8.3321608736E-3f) * z - 1.6666654611E-1f) * z * x + x;
}
static float cos_poly(float z) {
    return ((2.443315711809948E-005f * z - 1.388731625493765E-003f) * z + 4.166664568298827E-002f) * z * z
           - 0.5f * z + 1.0f;
}
#define FOPI 1.27323954473516f
#define DP1  0.78515625f
#define DP2  2.4187564849853515625e-4f
#define DP3  3.77489497744594108e-8f

float oracle_sinf(float xx) {
    float x = xx;
    int sgn = 0;
    if (x < 0.0f) { sgn = 1; x = -x; }
    if (!(x < 8192.0f)) { return (x == x) ? 0.0f : x; }   /* out of the reduction's range (never hit) */
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

float oracle_cosf(float xx) {
    float x = absf(xx);
    if (!(x < 8192.0f)) { return (x == x) ? 1.0f : x; }
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

/* 2^n for integer n, exactly, in two steps so that subnormal results round once per step. */
static float ldexp_(float y, int n) {
    if (n > 127) { y = y * bits_f(0x7F000000u); n -= 127; if (n > 127) n = 127; }
    if (n < -126) { y = y * bits_f(0x00800000u); n += 126; if (n < -126) n = -126; }
    return y * bits_f((uint32_t)(n + 127) << 23);
}

float oracle_expf(float x) {
    if (x != x) return x;
    if (x > 88.72283905206835f) return INFINITY;
    if (x < -103.278929903431851103f) return 0.0f;
    float z = floorf(1.44269504088896341f * x + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    z = x * x;
    float y = ((((( 1.9875691500E-4f * x + 1.3981999507E-3f) * x + 8.3334519073E-3f) * x
                 + 4.1665795894E-2f) * x + 1.6666665459E-1f) * x + 5.0000001201E-1f) * z + x + 1.0f;
    return ldexp_(y, n);
}

float oracle_logf(float x) {
    if (x != x) return x;
    if (x <= 0.0f) return x == 0.0f ? -INFINITY : NAN;
    if (x == INFINITY) return x;
    uint32_t u = f_bits(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 16777216.0f; e = -24; u = f_bits(x); }
    e += (int)((u >> 23) & 0xFFu) - 126;
    x = bits_f((u & 0x807FFFFFu) | 0x3F000000u);        /* mantissa in [0.5, 1) */
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

static float atanf_(float xx) {
    float x = xx;
    int sgn = 0;
    if (x < 0.0f) { sgn = 1; x = -x; }
    float y;
    if (x > 2.414213562373095f) { y = 1.5707963267948966192f; x = -(1.0f / x); }
    else if (x > 0.4142135623730950f) { y = 0.7853981633974483096f; x = (x - 1.0f) / (x + 1.0f); }
    else { y = 0.0f; }
    float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032E-1f) * z + 1.99777106478E-1f) * z
              - 3.33329491539E-1f) * z * x + x);
    return sgn ? -y : y;
}

float oracle_atan2f(float y, float x) {
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
    return w + atanf_(y / x);
}

float oracle_asinf(float xx) {
    float a = absf(xx);
    if (a > 1.0f) return NAN;
    if (a < 1.0e-4f) return xx;
    float x, z;
    int flag;
    if (a > 0.5f) { z = 0.5f * (1.0f - a); x = sqrtf(z); flag = 1; }
    else { x = a; z = x * x; flag = 0; }
    z = (((( 4.2163199048E-2f * z + 2.4181311049E-2f) * z + 4.5470025998E-2f) * z
          + 7.4953002686E-2f) * z + 1.6666752422E-1f) * z * x + x;
    if (flag) { z = z + z; z = 1.5707963267948966192f - z; }
    return xx < 0.0f ? -z : z;
}


/* Math mode: 0 = the deterministic spec above (bit-comparable with the HIP
 * kernels); 1 = the C library's sinf/cosf/expf/atan2f/asinf/powf, i.e. what the
 * reference itself calls.  Mode 1 is used to pin the oracle against the
 * reference's own observed outputs. */
static int g_libm = 0;
void oracle_set_math_mode(int libm) { g_libm = libm != 0; }
static inline float sinf_(float x) { return g_libm ? sinf(x) : oracle_sinf(x); }
static inline float cosf_(float x) { return g_libm ? cosf(x) : oracle_cosf(x); }
static inline float expf_(float x) { return g_libm ? expf(x) : oracle_expf(x); }
static inline float atan2f_(float y, float x) { return g_libm ? atan2f(y, x) : oracle_atan2f(y, x); }
static inline float asinf_(float x) { return g_libm ? asinf(x) : oracle_asinf(x); }
static inline float powf_(float x, float y) { return g_libm ? powf(x, y) : oracle_expf(y * oracle_logf(x)); }

/* ====================================================================== */
/* RNG (RT/samplers.h:3-108)                                              */
/* ====================================================================== */

typedef struct { uint32_t e[4]; } RandomSeries;

uint32_t oracle_wang_hash(uint32_t key) {                /* RT/samplers.h:3-12 */
    key += ~(key << 15);
    key ^=  (key >> 10);
    key +=  (key << 3);
    key ^=  (key >> 6);
    key += ~(key << 11);
    key ^=  (key >> 16);
    return key;
}
#define wang_hash oracle_wang_hash

static inline uint32_t hash_coordinate3(uint32_t x, uint32_t y, uint32_t z) {   /* RT/samplers.h:14-18 */
    return (x*73856093u) ^ (y*83492791u) ^ (z*871603259u);
}
static inline uint32_t hash_coordinate2(uint32_t x, uint32_t y) {               /* RT/samplers.h:20-27 */
    uint32_t qx = 1103515245u*((x >> 1) ^ y);
    uint32_t qy = 1103515245u*((y >> 1) ^ x);
    return 1103515245u*(qx ^ (qy >> 3));
}
static inline void next_set(RandomSeries* s, uint32_t out[4]) {                 /* RT/samplers.h:36-45 */
    for (int i = 0; i < 4; ++i) {
        uint32_t r = s->e[i];
        r ^= r << 13;
        r ^= r >> 17;
        r ^= r << 5;
        s->e[i] = r;
        out[i] = r;
    }
}
static inline void random_unilaterals(RandomSeries* s, float out[4]) {          /* RT/samplers.h:68-83 */
    uint32_t b[4];
    next_set(s, b);
    for (int i = 0; i < 4; ++i) out[i] = bits_f((127u << 23) | (b[i] >> 9)) - 1.0f;
}
static inline void random_bilaterals(RandomSeries* s, float out[4]) {           /* RT/samplers.h:85-90 */
    random_unilaterals(s, out);
    for (int i = 0; i < 4; ++i) out[i] = out[i]*2.0f - 1.0f;
}
static RandomSeries random_seed(uint32_t seed) {                                /* RT/samplers.h:92-108 */
    RandomSeries r;
    if (seed == 0) seed = 0xFFFFFFFFu;
    uint32_t h = wang_hash(seed);
    r.e[0] = r.e[1] = r.e[2] = r.e[3] = h;
    uint32_t a[4], b[4], c[4], d[4];
    next_set(&r, a); next_set(&r, b); next_set(&r, c); next_set(&r, d);
    r.e[0] = wang_hash(a[0]);
    r.e[1] = wang_hash(b[1]);
    r.e[2] = wang_hash(c[2]);
    return r;
}

/* Per-sample seed (RT_RNG_PER_SAMPLE): the reference's tile seed
 * (RT/raytracer.cpp:588-590) further keyed by pixel and sample index. */
uint32_t oracle_sample_seed(uint32_t total_frame_index, uint32_t frame_count, uint32_t tile_index,
                            uint32_t pixel_id, uint32_t canonical_sample_index) {
    uint32_t tile_seed = hash_coordinate3(total_frame_index, frame_count, tile_index);
    return wang_hash(tile_seed ^ wang_hash((pixel_id * 0x9E3779B9u) ^ wang_hash(canonical_sample_index + 0x68E31DA4u)));
}

void oracle_rng_unilaterals(uint32_t seed, uint32_t count, float* out) {
    RandomSeries s = random_seed(seed);
    for (uint32_t i = 0; i < count; ++i) random_unilaterals(&s, out + 4*i);
}

/* ====================================================================== */
/* Samplers (RT/samplers.cpp:18-138)                                      */
/* ====================================================================== */

enum { Sample_DirectLighting, Sample_IndirectLighting, Sample_LightSelection, Sample_Reflectance,
       Sample_DOF, Sample_AA, Sample_Roulette };                               /* RT/samplers.h:129-138 */

extern const unsigned char rt_strata_permutation_sets[256*64];   /* data/strata_permutation_sets.u8 */
extern const unsigned char rt_bluenoise_256spp[327680];          /* data/bluenoise_256spp.u8 */

typedef struct {
    RandomSeries* entropy;
    int strategy;
    uint32_t sample_index;
    uint32_t x, y;
} Sampler;                                                                      /* RT/samplers.h:140-145 */

/* samplerBlueNoiseErrorDistribution_128x128_OptimizedFor_2d2d2d2d_256spp
 * (RT/blue_noise_samplers/...256spp.cpp:14-34) over the u8 tables. */
static float blue_noise_256spp(int pixel_i, int pixel_j, int sample_index, int dim) {
    const unsigned char* sobol = rt_bluenoise_256spp;
    const unsigned char* scrambling = rt_bluenoise_256spp + 65536;
    const unsigned char* ranking = rt_bluenoise_256spp + 65536 + 131072;
    pixel_i &= 127; pixel_j &= 127; sample_index &= 255; dim &= 255;
    int ranked = sample_index ^ ranking[dim + (pixel_i + pixel_j*128)*8];
    int value = sobol[dim + ranked*256];
    value = value ^ scrambling[(dim % 8) + (pixel_i + pixel_j*128)*8];
    return (float)value / 256.0f;
}

static V2 get_next_sample_2d(Sampler* sampler, int dimension, uint32_t bounce_index) {   /* :18-90 */
    int strategy = sampler->strategy;
    uint32_t x = sampler->x, y = sampler->y, index = sampler->sample_index;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && index > 256) strategy = RT_SAMPLING_STRATIFIED;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && dimension >= 4) strategy = RT_SAMPLING_STRATIFIED;
    V2 sample = { 0, 0 };
    float u[4];
    if (bounce_index == 0) {
        if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE) {
            random_unilaterals(sampler->entropy, u);
            float ex = (1.0f / 256.0f)*u[0], ey = (1.0f / 256.0f)*u[1];
            sample.x = ex + blue_noise_256spp((int)x, (int)y, (int)index, 2*dimension);
            sample.y = ey + blue_noise_256spp((int)x, (int)y, (int)index, 2*dimension + 1);
        } else if (strategy == RT_SAMPLING_STRATIFIED) {
            const float rx = 1.0f / 8.0f, ry = 1.0f / 8.0f;
            uint32_t index_offset = (73856093u*(uint32_t)dimension) ^ hash_coordinate2(x, y);
            uint32_t si = rt_strata_permutation_sets[(index_offset & 255u)*64u + (index % 64u)];
            float sx = (float)(si % 8u)*rx, sy = (float)(si / 8u)*ry;
            random_unilaterals(sampler->entropy, u);
            float ox = u[0]*rx, oy = u[1]*ry;
            sample.x = sx + ox; sample.y = sy + oy;
        } else {
            random_unilaterals(sampler->entropy, u);
            sample.x = u[0]; sample.y = u[1];
        }
    } else {
        random_unilaterals(sampler->entropy, u);
        sample.x = u[0]; sample.y = u[1];
    }
    return sample;
}

static float get_next_sample_1d(Sampler* sampler, int dimension, uint32_t bounce_index) {  /* :92-138 */
    int strategy = sampler->strategy;
    uint32_t x = sampler->x, y = sampler->y, index = sampler->sample_index;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && index > 256) strategy = RT_SAMPLING_STRATIFIED;
    if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE && dimension >= 4) strategy = RT_SAMPLING_STRATIFIED;
    float u[4];
    float sample;
    if (bounce_index == 0) {
        if (strategy == RT_SAMPLING_OPTIMIZED_BLUE_NOISE) {
            random_unilaterals(sampler->entropy, u);
            float e = (1.0f / 256.0f)*u[0];
            sample = e + blue_noise_256spp((int)x, (int)y, (int)index, 2*dimension);
        } else if (strategy == RT_SAMPLING_STRATIFIED) {
            const float rc = 1.0f / 64.0f;
            uint32_t index_offset = (73856093u*(uint32_t)dimension) ^ hash_coordinate2(x, y);
            uint32_t si = rt_strata_permutation_sets[(index_offset & 255u)*64u + (index % 64u)];
            float strata = (float)si*rc;
            random_unilaterals(sampler->entropy, u);
            float offset = u[0]*rc;
            sample = strata + offset;
        } else {
            random_unilaterals(sampler->entropy, u);
            sample = u[0];
        }
    } else {
        random_unilaterals(sampler->entropy, u);
        sample = u[0];
    }
    return sample;
}

void oracle_sample_2d(uint32_t seed, int strategy, uint32_t x, uint32_t y, uint32_t index,
                      int dimension, uint32_t bounce, float* out2) {
    RandomSeries e = random_seed(seed);
    Sampler s = { &e, strategy, index, x, y };
    V2 r = get_next_sample_2d(&s, dimension, bounce);
    out2[0] = r.x; out2[1] = r.y;
}
float oracle_sample_1d(uint32_t seed, int strategy, uint32_t x, uint32_t y, uint32_t index,
                       int dimension, uint32_t bounce) {
    RandomSeries e = random_seed(seed);
    Sampler s = { &e, strategy, index, x, y };
    return get_next_sample_1d(&s, dimension, bounce);
}

/* ====================================================================== */
/* Intersection (RT/intersection.h:5-24, RT/intersection.cpp:12-610)      */
/* ====================================================================== */

typedef struct {
    V3 o, d, inv_d;
    int neg[3];
    float max_t;
} Ray;

static inline Ray make_ray(V3 o, V3 d, float far_clip) {     /* RT/intersection.h:13-24 */
    Ray r;
    r.o = o; r.d = d;
    r.inv_d = sdiv(1.0f, d);
    r.neg[0] = d.x < 0.0f; r.neg[1] = d.y < 0.0f; r.neg[2] = d.z < 0.0f;
    r.max_t = far_clip;
    return r;
}

static inline int ray_intersect_plane(const Ray* ray, V3 n, float d, float* out_t) { /* :12-42 */
    float denom = dot(n, ray->d);
    if (denom < -EPSILON) {
        float t = (d - dot(n, ray->o)) / denom;
        if ((t >= EPSILON) && (t < *out_t)) { *out_t = t; return 1; }
    }
    return 0;
}

static inline int ray_intersect_sphere(const Ray* ray, float r, float* out_t) {       /* :44-74 */
    V3 o = ray->o;
    float r_sq = r*r;
    float b = dot(ray->d, o);
    float c = dot(o, o) - r_sq;
    float discr = (b*b - c);
    if (discr >= 0) {
        float root = sqrtf(discr);
        float tn = -b - root;
        float tf = -b + root;
        float t = (tn >= 0.0f ? tn : tf);
        if ((t >= EPSILON) && (*out_t > t)) { *out_t = t; return 1; }
    }
    return 0;
}

static inline int ray_intersect_box(const Ray* ray, V3 box_r, float* out_t) {          /* :76-105 */
    V3 m = ray->inv_d;
    V3 n = mul(m, ray->o);
    V3 k = mul(vabs(m), box_r);
    V3 t1 = sub(neg(n), k);
    V3 t2 = add(neg(n), k);
    float tn = mx(mx(t1.x, t1.y), t1.z);
    float tf = mn(mn(t2.x, t2.y), t2.z);
    if (tn < tf) {
        float t = (tn >= 0.0f ? tn : tf);
        if ((*out_t > t) && (t >= EPSILON)) { *out_t = t; return 1; }
    }
    return 0;
}

static inline int ray_intersect_bv(const Ray* ray, V3 p, V3 r, float far_clip) {       /* :107-133 */
    V3 rel = sub(ray->o, p);
    V3 m = ray->inv_d;
    V3 n = mul(m, rel);
    V3 k = mul(vabs(m), r);
    V3 t1 = sub(neg(n), k);
    V3 t2 = add(neg(n), k);
    float tn = mx(mx(t1.x, t1.y), t1.z);
    float tf = mn(mn(t2.x, t2.y), t2.z);
    return ((tn < tf) && (tf > 0.0f)) && (tn < far_clip);
}

static inline int ray_intersect_triangle(const Ray* ray, V3 a, V3 b, V3 c,
                                         float* out_t, V3* out_uvw) {                  /* :135-182 */
    const float eps = 0.000000001f;
    V3 e1 = sub(b, a);
    V3 e2 = sub(c, a);
    V3 pvec = cross(ray->d, e2);
    float det = dot(e1, pvec);
    if (det > -eps && det < eps) return 0;
    float inv_det = 1.0f / det;
    V3 tvec = sub(ray->o, a);
    float v = dot(tvec, pvec)*inv_det;
    if (v < 0.0f || v > 1.0f) return 0;
    V3 qvec = cross(tvec, e1);
    float w = dot(ray->d, qvec)*inv_det;
    if (w < 0.0f || v + w > 1.0f) return 0;
    float t = dot(e2, qvec)*inv_det;
    if ((t < eps) || (*out_t < t)) return 0;
    *out_t = t;
    *out_uvw = v3(1.0f - v - w, v, w);
    return 1;
}

/* TraversalStats (RT/intersection.h:33-40) as the reference counts them: TS_CALLS per intersect_mesh
   call (RT/intersection.cpp:254); per traversal the nodes taken from the stack (:274), the interior
   ones (:358) and the leaves (:279) that pass their pop-time test, added when the traversal ends
   (:378-380) -- not when an occlusion query returns from inside it (:297-299). */
enum { TS_CALLS, TS_BVH, TS_NODES, TS_LEAVES, TS_N };

/* The GPU walk's counts per query kind (gpu_walk_query below): mesh instances reached (the GPU's
   mesh_intersection_count), entered (its entry steps), leaves entered (mesh_leaf_traversals), BVH4
   interior nodes expanded (mesh_node_traversals: the BVH2 interior nodes at even depth below a mesh
   root, which are the BVH4's), triangle steps (up to TRI_FETCH = 2 triangles per step; the GPU's
   mesh_bvh_traversals = entries + nodes + triangle steps). */
enum { GW_CALLS, GW_ENTRIES, GW_LEAVES, GW_NODES4, GW_TRISTEPS, GW_N };

/* The GPU's degenerate-axis pruning (bv_static in buas-pathtracer_amd/csrc/rt_kernels.hip, mesh BVHs
   only): for a ray with a direction component exactly 0, a node whose slab on that axis excludes the
   ray's coordinate by more than 1 % of the node's largest half extent plus 1e-5 of its position is
   skipped (it holds no triangle the ray can hit; the reference's NaN slab keeps it).  The results are
   the reference's either way; only the GPU walk's node and leaf counts see it. */
static inline int gpu_pruned(const Ray* ray, V3 p, V3 r) {
    const int zx = ray->d.x == 0.0f, zy = ray->d.y == 0.0f, zz = ray->d.z == 0.0f;
    if (!(zx || zy || zz)) return 0;
    const V3 rel = sub(ray->o, p);
    const float margin = 0.01f*mx(r.x, mx(r.y, r.z)) + 1e-5f*mx(fabsf(p.x), mx(fabsf(p.y), fabsf(p.z)));
    return (zx && fabsf(rel.x) > r.x + margin) || (zy && fabsf(rel.y) > r.y + margin) ||
           (zz && fabsf(rel.z) > r.z + margin);
}

/* intersect_mesh, BVHStorage_Scalar path (RT/intersection.cpp:243-401).  ts: the reference's
   TraversalStats of the query kind (or NULL); gw: the GPU walk's counts (GW_*, gpu_walk_query below;
   or NULL), counted whether or not the traversal returns early, in which case the walk also applies
   the GPU's degenerate-axis pruning (gpu_pruned).  The stack entries carry their depth's parity in
   bit 31 (the BVH4 nodes are the even-depth interior ones). */
static int intersect_mesh(const rt_mesh* mesh, const Ray* ray, int occlusion, float* out_t,
                          uint32_t* out_tri, V3* out_uvw, V3* out_a, V3* out_b, V3* out_c,
                          uint64_t* ts, uint64_t* gw) {
    uint32_t hit_tri = 0xFFFFFFFFu;
    uint32_t stack[64];
    uint32_t at = 0;
    uint64_t trav = 0, nodes = 0, leaves = 0, nodes4 = 0, tristeps = 0;
    if (ts) ts[TS_CALLS]++;
    if (!mesh->node_count || !mesh->nodes) return 0;            /* `if (bvh)` (:259): no BVH, no triangle */
    stack[at++] = 0;
    while (at > 0) {
        const uint32_t e = stack[--at], odd = e >> 31;
        const rt_bvh_node* node = &mesh->nodes[e & 0x7FFFFFFFu];
        ++trav;
        if (ray_intersect_bv(ray, node->bv_p, node->bv_r, *out_t) &&
            !(gw && gpu_pruned(ray, node->bv_p, node->bv_r))) {
            if (node->count) {
                ++leaves;
                uint32_t first = node->left_first;
                for (uint32_t i = 0; i < node->count; ++i) {
                    const rt_v3* tri = &mesh->triangles[3*(size_t)(first + i)];
                    if (ray_intersect_triangle(ray, tri[0], tri[1], tri[2], out_t, out_uvw)) {
                        if (occlusion) {
                            if (gw) {
                                gw[GW_LEAVES] += leaves; gw[GW_NODES4] += nodes4;
                                gw[GW_TRISTEPS] += tristeps + i/2 + 1;       /* the step holding triangle i */
                            }
                            return 1;
                        }
                        *out_a = tri[0]; *out_b = tri[1]; *out_c = tri[2];
                        hit_tri = mesh->indices[first + i];
                    }
                }
                tristeps += (node->count + 1)/2;
            } else {
                ++nodes;
                if (!odd) ++nodes4;
                uint32_t left = node->left_first;
                const uint32_t d = (odd ^ 1u) << 31;
                if (at + 2 > 64) return 0;    /* the reference overflows its stack[64] here (UB) */
                if (ray->neg[node->split_axis]) { stack[at++] = left | d; stack[at++] = (left + 1) | d; }
                else { stack[at++] = (left + 1) | d; stack[at++] = left | d; }
            }
        }
    }
    if (ts) { ts[TS_BVH] += trav; ts[TS_NODES] += nodes; ts[TS_LEAVES] += leaves; }
    if (gw) { gw[GW_LEAVES] += leaves; gw[GW_NODES4] += nodes4; gw[GW_TRISTEPS] += tristeps; }
    if (hit_tri != 0xFFFFFFFFu) { *out_tri = hit_tri; return 1; }
    return 0;
}

static inline Ray transform_ray(const Ray* ray, const rt_m4x4* m) {   /* :403-409 */
    V3 o = xform(m, ray->o, 1.0f);
    V3 d = xform(m, ray->d, 0.0f);
    return make_ray(o, d, ray->max_t);
}

typedef struct {
    int hit;            /* 0 miss, 1 plane, 2 primitive */
    uint32_t index;     /* plane index or primitive index */
    float t;
    V3 hit_p, n;
} Hit;

/* intersect_scene_internal (RT/intersection.cpp:411-598).  Returns 1 on hit.  ts: TraversalStats
   of the query kind (TS_*), or NULL. */
static int intersect_scene_internal(const rt_scene_desc* scene, const Ray* ray, int occlusion,
                                    uint32_t ignored, Hit* out, uint64_t* ts) {
    float t = ray->max_t;
    int hit_kind = 0;
    uint32_t hit_index = 0;
    for (uint32_t i = 0; i < scene->plane_count; ++i) {
        const rt_primitive* pl = &scene->planes[i];
        if (ray_intersect_plane(ray, v3(pl->p[0], pl->p[1], pl->p[2]), pl->p[3], &t)) {
            hit_kind = 1; hit_index = i;
        }
    }
    uint32_t hit_tri = 0;
    V3 a = {0,0,0}, b = {0,0,0}, c = {0,0,0}, uvw = {0,0,0};
    Ray os_ray;
    memset(&os_ray, 0, sizeof(os_ray));
    if (scene->bvh_node_count) {
        uint32_t stack[64];
        uint32_t at = 0;
        stack[at++] = 0;
        while (at > 0) {
            const rt_bvh_node* node = &scene->bvh_nodes[stack[--at]];
            if (ray_intersect_bv(ray, node->bv_p, node->bv_r, t)) {
                if (node->count) {
                    for (uint32_t li = 0; li < node->count; ++li) {
                        uint32_t pi = scene->bvh_indices[node->left_first + li];
                        if (pi == ignored) continue;
                        const rt_primitive* prim = &scene->primitives[pi];
                        Ray ir = transform_ray(ray, &scene->transforms[prim->transform_index].inverse);
                        int hit_any = 0;
                        switch (prim->type) {
                            case RT_PRIMITIVE_SPHERE: hit_any = ray_intersect_sphere(&ir, prim->p[0], &t); break;
                            case RT_PRIMITIVE_BOX: hit_any = ray_intersect_box(&ir, v3(prim->p[0], prim->p[1], prim->p[2]), &t); break;
                            case RT_PRIMITIVE_MESH:
                                hit_any = intersect_mesh(&scene->meshes[prim->mesh_index], &ir, occlusion, &t,
                                                         &hit_tri, &uvw, &a, &b, &c, ts, NULL);
                                break;
                            default: break;
                        }
                        if (hit_any) {
                            if (occlusion) { out->hit = 2; out->index = pi; out->t = t; return 1; }
                            hit_kind = 2; hit_index = pi; os_ray = ir;
                        }
                    }
                } else {
                    uint32_t left = node->left_first;
                    if (at + 2 > 64) break;
                    if (ray->neg[node->split_axis]) { stack[at++] = left; stack[at++] = left + 1; }
                    else { stack[at++] = left + 1; stack[at++] = left; }
                }
            }
        }
    }
    out->hit = hit_kind;
    out->index = hit_index;
    out->t = t;
    if (hit_kind && !occlusion) {                                 /* :NormalCalculation :526-591 */
        V3 os_p = add(os_ray.o, smul(t, os_ray.d));
        out->hit_p = add(ray->o, smul(t, ray->d));
        V3 n = {0,0,0};
        const rt_m4x4* inv;
        if (hit_kind == 1) {
            const rt_primitive* pl = &scene->planes[hit_index];
            n = v3(pl->p[0], pl->p[1], pl->p[2]);
            inv = &scene->transforms[pl->transform_index].inverse;
        } else {
            const rt_primitive* prim = &scene->primitives[hit_index];
            inv = &scene->transforms[prim->transform_index].inverse;
            if (prim->type == RT_PRIMITIVE_SPHERE) {
                n = os_p;
            } else if (prim->type == RT_PRIMITIVE_BOX) {
                V3 rel = divv(os_p, v3(prim->p[0], prim->p[1], prim->p[2]));
                int li = 0;
                float le = absf(rel.x);
                if (absf(rel.y) > le) { li = 1; le = absf(rel.y); }
                if (absf(rel.z) > le) { li = 2; le = absf(rel.z); }
                float s = sign_of(comp(rel, li));
                n = v3(li == 0 ? s : 0.0f, li == 1 ? s : 0.0f, li == 2 ? s : 0.0f);
            } else if (prim->type == RT_PRIMITIVE_MESH) {
                const rt_mesh* mesh = &scene->meshes[prim->mesh_index];
                if (mesh->has_normals) {
                    const rt_v3* nt = &mesh->normals[3*(size_t)hit_tri];
                    n = add(add(smul(uvw.x, nt[0]), smul(uvw.y, nt[1])), smul(uvw.z, nt[2]));
                } else {
                    V3 e1 = normalize(sub(b, a));
                    V3 e2 = normalize(sub(c, a));
                    n = cross(e1, e2);
                }
            }
        }
        out->n = noz(xform_normal(inv, n));
    }
    return hit_kind != 0;
}

/* ---------------------------------------------------------------------- */
/* The MI355X library's walk, restated for its TraversalStats (rt_stats::traversal on the GPU;
   DESIGN.md section 3).  Not the reference: the GPU tests the planes and the top level's spheres and
   boxes before any mesh BVH (ray_prologue in buas-pathtracer_amd/csrc/rt_kernels.hip), so the mesh
   instances it reaches and enters and the leaves it visits are counted in that order:
     - the prologue walks the top level in one fixed order (octant 0: the left child first) with t
       from the planes and the analytic primitives only; a mesh instance whose leaf passes is reached
       (GW_CALLS: the GPU's mesh_intersection_count), and listed when its root box passes at that t;
       an analytic occluder ends a shadow query there;
     - a query with 1..mlist_max listed instances enters them in list order (GW_ENTRIES), each with
       its BVH walked from the current t (GW_LEAVES: leaves taken from the stack with their far-clip
       test passed), a shadow query ending at the first occluding instance;
     - a query with more (MLIST_FULL), or every query of a scene whose top level is too large for the
       prologue, walks the whole top level from the root in the reference's front-to-back order,
       starting at the prologue's t, entering every mesh instance whose leaf passes (for the scene
       whose top level is too large, these entries are the GPU's mesh_intersection_count).
   The leaves are the BVH4's (the BVH2's leaves, which it visits in the BVH2's depth-first order),
   walked here in the BVH2's front-to-back order with the GPU's pruning of nodes that a ray with an
   exactly-zero direction component cannot hit (gpu_pruned), so the GPU's leaf counts equal these
   up to float ties (a few leaves in 10^7 on C3 and C4 at 480x270).  GW_CALLS is exact. */
/* (GW_* counters: defined before intersect_mesh) */
static int g_gw_on = 0;
static uint32_t g_gw_mlist = 4;
static int g_gw_top = 1;
static uint64_t g_gw_acc[2][GW_N];
static pthread_mutex_t g_gw_mu = PTHREAD_MUTEX_INITIALIZER;

void oracle_gpu_walk_stats(int on, uint32_t mlist_max, int top_prologue) {
    pthread_mutex_lock(&g_gw_mu);
    g_gw_on = on != 0;
    g_gw_mlist = mlist_max;
    g_gw_top = top_prologue != 0;
    memset(g_gw_acc, 0, sizeof(g_gw_acc));
    pthread_mutex_unlock(&g_gw_mu);
}

void oracle_gpu_walk_result(uint64_t out[2*GW_N]) {
    pthread_mutex_lock(&g_gw_mu);
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < GW_N; ++i) out[k*GW_N + i] = g_gw_acc[k][i];
    pthread_mutex_unlock(&g_gw_mu);
}

static void gw_add(const uint64_t g[2][GW_N]) {
    if (!g_gw_on) return;
    pthread_mutex_lock(&g_gw_mu);
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < GW_N; ++i) g_gw_acc[k][i] += g[k][i];
    pthread_mutex_unlock(&g_gw_mu);
}

/* a mesh instance entered by the trace kernel: its object-space ray, its BVH from t */
static int gw_mesh(const rt_scene_desc* sc, const rt_primitive* prim, const Ray* ray, int occ, float* t,
                   uint64_t* g) {
    Ray ir = transform_ray(ray, &sc->transforms[prim->transform_index].inverse);
    uint32_t tri;
    V3 uvw, a, b, c;
    g[GW_ENTRIES]++;
    return intersect_mesh(&sc->meshes[prim->mesh_index], &ir, occ, t, &tri, &uvw, &a, &b, &c, NULL, g);
}

/* the top level walked with `neg` as the direction signs (the reference's order for the ray's own, the
   prologue's for 0); list != NULL: the prologue (spheres and boxes tested, mesh instances reached, and
   listed when their root box passes); NULL: the trace kernel (mesh instances entered, and counted as
   reached when `calls`).  Returns 1 when a shadow query is occluded. */
static int gw_top(const rt_scene_desc* sc, const Ray* ray, const int neg[3], int occ, uint32_t ignored, float* t,
                  uint32_t* list, uint32_t* n, uint64_t* g, int calls) {
    uint32_t stack[64];
    uint32_t at = 0;
    stack[at++] = 0;
    while (at > 0) {
        const rt_bvh_node* node = &sc->bvh_nodes[stack[--at]];
        if (!ray_intersect_bv(ray, node->bv_p, node->bv_r, *t)) continue;
        if (node->count) {
            for (uint32_t li = 0; li < node->count; ++li) {
                const uint32_t pi = sc->bvh_indices[node->left_first + li];
                if (pi == ignored) continue;
                const rt_primitive* prim = &sc->primitives[pi];
                Ray ir = transform_ray(ray, &sc->transforms[prim->transform_index].inverse);
                int hit = 0;
                if (prim->type == RT_PRIMITIVE_SPHERE) hit = ray_intersect_sphere(&ir, prim->p[0], t);
                else if (prim->type == RT_PRIMITIVE_BOX) hit = ray_intersect_box(&ir, v3(prim->p[0], prim->p[1], prim->p[2]), t);
                else if (prim->type == RT_PRIMITIVE_MESH) {
                    if (list || calls) g[GW_CALLS]++;
                    if (list) {
                        const rt_bvh_node* root = &sc->meshes[prim->mesh_index].nodes[0];
                        if (ray_intersect_bv(&ir, root->bv_p, root->bv_r, *t) && !gpu_pruned(&ir, root->bv_p, root->bv_r)) {
                            if (*n < 64) list[*n] = pi;
                            ++*n;
                        }
                    } else {
                        hit = gw_mesh(sc, prim, ray, occ, t, g);
                    }
                }
                if (hit && occ) return 1;
            }
        } else {
            const uint32_t left = node->left_first;
            if (at + 2 > 64) break;
            if (neg[node->split_axis]) { stack[at++] = left; stack[at++] = left + 1; }
            else { stack[at++] = left + 1; stack[at++] = left; }
        }
    }
    return 0;
}

/* Whether the library's ray prologue walks this top level: top_sequences (rt_kernels.hip) builds
 * its per-octant sequences only for at most 255 nodes and 63 bvh_indices slots, and gives up on a
 * node index out of range, a walk deeper than 64, or a leaf of more than 127 primitives or past the
 * slots; then the trace kernels walk the whole top level.  The same checks, on octant 0's order
 * (every octant visits the same nodes). */
static int gw_top_node_ok(const rt_scene_desc* sc, uint32_t n, uint32_t depth) {
    if (n >= sc->bvh_node_count || depth > 64) return 0;
    const rt_bvh_node* nd = &sc->bvh_nodes[n];
    if (nd->count) return nd->count <= 127 && nd->left_first + nd->count <= sc->bvh_index_count;
    if (nd->left_first == 0 || nd->left_first + 1 >= sc->bvh_node_count || nd->split_axis > 2) return 1;
    return gw_top_node_ok(sc, nd->left_first, depth + 1) && gw_top_node_ok(sc, nd->left_first + 1, depth + 1);
}
static int gw_top_prologue(const rt_scene_desc* sc) {
    return sc->bvh_node_count && sc->bvh_node_count <= 255 && sc->bvh_index_count <= 63 && gw_top_node_ok(sc, 0, 0);
}

static void gpu_walk_query(const rt_scene_desc* sc, const Ray* ray, int occ, uint32_t ignored, uint64_t* g) {
    float t = ray->max_t;
    for (uint32_t i = 0; i < sc->plane_count; ++i) {                  /* the planes first */
        const rt_primitive* pl = &sc->planes[i];
        if (ray_intersect_plane(ray, v3(pl->p[0], pl->p[1], pl->p[2]), pl->p[3], &t) && occ) return;
    }
    if (!sc->bvh_node_count) return;
    /* the prologue walks the top level when it fits its tables (top_sequences, rt_kernels.hip) */
    if (g_gw_top && gw_top_prologue(sc)) {
        static const int oct0[3] = {0, 0, 0};
        uint32_t list[64], n = 0;
        if (gw_top(sc, ray, oct0, occ, ignored, &t, list, &n, g, 0)) return;
        if (n == 0) return;                                            /* not queued */
        if (n <= g_gw_mlist) {
            for (uint32_t k = 0; k < n; ++k)
                if (gw_mesh(sc, &sc->primitives[list[k]], ray, occ, &t, g) && occ) return;
            return;
        }
        (void)gw_top(sc, ray, ray->neg, occ, ignored, &t, NULL, NULL, g, 0);   /* MLIST_FULL: the kernel walks */
        return;
    }
    const rt_bvh_node* root = &sc->bvh_nodes[0];
    if (!ray_intersect_bv(ray, root->bv_p, root->bv_r, t)) return;
    (void)gw_top(sc, ray, ray->neg, occ, ignored, &t, NULL, NULL, g, 1);      /* the kernel's walk reaches them */
}

/* ====================================================================== */
/* Integrator (RT/integrators.cpp)                                        */
/* ====================================================================== */

/* Environment-map sampling table (oracle_set_env_sampling; rt_set_env_sampling in
   include/rt_abi.h).  Beyond the reference: load_environment_map builds a tile luma CDF
   (RT/assets.cpp:620-665) that nothing reads (RT/integrators.cpp:230-233).  The tiles are
   that CDF's grid; the table is the alias form of the same tile sums. */
typedef struct {
    uint32_t n, tx, tw, th;
    float* prob;          /* alias threshold */
    uint32_t* alias;
    float* dens;          /* tile probability x texels / tile texels: pdf over the (u, v) square */
} EnvTab;

typedef struct {
    const rt_scene_desc* scene;
    const rt_settings* settings;
    const rt_material* air;
    uint64_t closest_rays, shadow_rays;
    const EnvTab* env;    /* NULL: the reference's estimator */
    uint64_t ts[2][TS_N]; /* TraversalStats per query kind: [0] intersect_scene, [1] intersect_shadow_ray */
    uint64_t gw[2][GW_N]; /* the GPU walk's counts (gpu_walk_query), when g_gw_on */
} Ctx;

static int g_env_sampling = 0;
void oracle_set_env_sampling(int mode) { g_env_sampling = mode != 0; }

static void env_tab_free(EnvTab* t) {
    free(t->prob); free(t->alias); free(t->dens);
    memset(t, 0, sizeof(*t));
}

/* tile luma sums in load_environment_map's order (RT/assets.cpp:634-656, luma RT/common.h:142),
   probabilities luma / total, Vose's alias construction (stacks popped from the end) */
static int env_tab_build(const rt_scene_desc* sc, EnvTab* t) {
    memset(t, 0, sizeof(*t));
    const uint32_t w = sc->skydome_w, h = sc->skydome_h;
    if (!sc->skydome || w < 32 || h < 32) return 0;
    t->tw = w / 32; t->th = h / 32;
    t->tx = (w + t->tw - 1) / t->tw;
    const uint32_t ty = (h + t->th - 1) / t->th, n = t->tx*ty;
    t->n = n;
    float* lum = (float*)malloc(sizeof(float)*n);
    float* scaled = (float*)malloc(sizeof(float)*n);
    uint32_t* small = (uint32_t*)malloc(sizeof(uint32_t)*n);
    uint32_t* large = (uint32_t*)malloc(sizeof(uint32_t)*n);
    t->prob = (float*)malloc(sizeof(float)*n);
    t->alias = (uint32_t*)malloc(sizeof(uint32_t)*n);
    t->dens = (float*)malloc(sizeof(float)*n);
    float sum = 0.0f;
    int ok = 1;
    for (uint32_t k = 0; k < n && ok; ++k) {
        uint32_t x0 = (k % t->tx)*t->tw, y0 = (k / t->tx)*t->th;
        uint32_t x1 = x0 + t->tw < w ? x0 + t->tw : w, y1 = y0 + t->th < h ? y0 + t->th : h;
        float cur = 0.0f;
        for (uint32_t y = y0; y < y1; ++y)
            for (uint32_t x = x0; x < x1; ++x) {
                const rt_v3* c = &sc->skydome[(size_t)y*w + x];
                cur += 0.299f*c->x + 0.587f*c->y + 0.114f*c->z;
            }
        if (!(cur >= 0.0f)) ok = 0;
        lum[k] = cur;
        sum += cur;
    }
    if (!ok || !(sum > 0.0f) || !isfinite(sum)) ok = 0;
    if (ok) {
        float rcp = 1.0f / sum;
        uint32_t ns = 0, nl = 0;
        for (uint32_t k = 0; k < n; ++k) {
            uint32_t x0 = (k % t->tx)*t->tw, y0 = (k / t->tx)*t->th;
            uint32_t cw = (x0 + t->tw < w ? x0 + t->tw : w) - x0, ch = (y0 + t->th < h ? y0 + t->th : h) - y0;
            float p = lum[k]*rcp;
            t->dens[k] = p*((float)((uint64_t)w*h) / (float)(cw*ch));
            scaled[k] = p*(float)n;
            t->prob[k] = 1.0f;
            t->alias[k] = k;
            if (scaled[k] < 1.0f) small[ns++] = k; else large[nl++] = k;
        }
        while (ns && nl) {
            uint32_t l = small[--ns], g = large[--nl];
            t->prob[l] = scaled[l];
            t->alias[l] = g;
            scaled[g] = (scaled[g] + scaled[l]) - 1.0f;
            if (scaled[g] < 1.0f) small[ns++] = g; else large[nl++] = g;
        }
    }
    free(lum); free(scaled); free(small); free(large);
    if (!ok) env_tab_free(t);
    return ok;
}

static V3 random_in_unit_sphere(RandomSeries* e) {            /* :11-19 */
    V3 r; float u[4];
    int guard = 0;   /* same bound as the device (an all-zero RandomSeries never terminates) */
    do { random_bilaterals(e, u); r = v3(u[0], u[1], u[2]); } while (length_sq(r) >= 1.0f && ++guard < 4096);
    return r;
}

static inline void get_tangents(V3 n, V3* b1, V3* b2) {        /* :58-66 */
    float sign = copy_sign(1.0f, n.z);
    float a = -1.0f / (sign + n.z);
    float b = n.x*n.y*a;
    *b1 = v3(1.0f + sign*n.x*n.x*a, sign*b, -sign*n.x);
    *b2 = v3(b, sign + n.y*n.y*a, -n.y);
}
static inline V3 oriented_around_normal(V3 v, V3 N) {          /* :68-75 */
    V3 T, B;
    get_tangents(N, &T, &B);
    return add(add(smul(v.x, B), smul(v.y, N)), smul(v.z, T));
}
static inline V3 map_to_hemisphere(V3 N, V2 rs) {              /* :93-105 */
    float az = TAU_32*rs.x, y = rs.y;
    V3 h;
    h.x = cosf_(az)*sqrtf(1.0f - y*y);
    h.y = y;
    h.z = sinf_(az)*sqrtf(1.0f - y*y);
    return oriented_around_normal(h, N);
}
static inline V3 map_to_cosine_weighted_hemisphere(V3 N, V2 rs) { /* :107-119 */
    float az = TAU_32*rs.x, y = rs.y;
    V3 h;
    h.x = cosf_(az)*sqrtf(1.0f - y);
    h.y = sqrtf(y);
    h.z = sinf_(az)*sqrtf(1.0f - y);
    return oriented_around_normal(h, N);
}

/* pick_random_light (:135-192); returns light primitive id, *out_p = pdf/sum */
static uint32_t pick_random_light(const Ctx* ctx, float rs, V3 I, float* out_rcp_pdf) {
    const rt_scene_desc* sc = ctx->scene;
    uint32_t n = sc->light_count;
    uint32_t result = 0;
    if (n > 0) {
        if (ctx->settings->importance_sample_lights) {
            float sum = 0.0f;
            float pdfs[256], cdf[256];
            float* P = n <= 256 ? pdfs : (float*)malloc(sizeof(float)*n);
            float* C = n <= 256 ? cdf : (float*)malloc(sizeof(float)*n);
            for (uint32_t i = 0; i < n; ++i) {
                const rt_primitive* light = &sc->primitives[sc->lights[i]];
                const rt_material* m = &sc->materials[light->material_id];
                V3 lv = sub(translation(&sc->transforms[light->transform_index].forward), I);
                float dsq = length_sq(lv);
                float l = max3(m->emission_color);
                float psa = 0.0f;
                if (light->type == RT_PRIMITIVE_SPHERE) {       /* projected_solid_angle :123-133 */
                    float r = light->p[0];
                    psa = PI_32*r*r / dsq;
                }
                float pdf = l*psa;
                sum += pdf;
                P[i] = pdf;
                float prev = (i > 0 ? C[i - 1] : 0.0f);
                C[i] = prev + pdf;
            }
            float e = sum*rs;
            uint32_t li = 0;
            while (li < n - 1 && C[li] < e) ++li;
            *out_rcp_pdf = P[li] / sum;
            result = sc->lights[li];
            if (P != pdfs) free(P);
            if (C != cdf) free(C);
        } else {
            *out_rcp_pdf = 1.0f / (float)n;
            float f = rs*(float)n - EPSILON;
            uint32_t li = f <= 0.0f ? 0u : (uint32_t)f;     /* (u32) of a float in (-1,0) truncates to 0 */
            if (li >= n) li = n - 1;
            result = sc->lights[li];
        }
    }
    return result;
}

typedef struct { V3 L, Nl; float dist, dist_sq, A; } LightSample;

static LightSample random_point_on_light(const Ctx* ctx, const rt_primitive* light, V2 rs, V3 I) { /* :199-228 */
    LightSample r;
    memset(&r, 0, sizeof(r));
    const rt_m4x4* fwd = &ctx->scene->transforms[light->transform_index].forward;
    V3 light_p = translation(fwd);
    V3 towards = normalize(sub(light_p, I));
    if (light->type == RT_PRIMITIVE_SPHERE) {
        float rad = light->p[0];
        V3 Nl = map_to_hemisphere(neg(towards), rs);
        V3 p = muls(Nl, rad);
        V3 pw = xform(fwd, p, 1.0f);
        V3 L = sub(pw, I);
        r.dist_sq = length_sq(L);
        r.dist = sqrtf(r.dist_sq);
        L = divs(L, r.dist);
        r.A = 2.0f*PI_32*rad*rad;
        r.L = L;
        r.Nl = Nl;
    }
    return r;
}

static inline float fresnel_dielectric(float cos_i, float eta_i, float eta_t, float eta_ratio,
                                       float* out_cos_t) {          /* :235-258 */
    float sin_i = sqrtf(mx(0.0f, 1.0f - cos_i*cos_i));
    float sin_t = eta_ratio*sin_i;
    float cos_t = sqrtf(mx(0.0f, 1.0f - sin_t*sin_t));
    *out_cos_t = cos_t;
    if (sin_t >= 1) return 1;
    float rpar = (((eta_t*cos_i) - (eta_i*cos_t)) / ((eta_t*cos_i) + (eta_i*cos_t)));
    float rperp = (((eta_i*cos_i) - (eta_t*cos_t)) / ((eta_i*cos_i) + (eta_t*cos_t)));
    return 0.5f * (rpar * rpar + rperp * rperp);
}

static inline V3 refract(V3 D, V3 N, float cos_i, float cos_t, float eta) {   /* :260-264 */
    return add(smul(eta, D), muls(N, (eta*cos_i - cos_t)));
}

static V3 sample_sky(const rt_scene_desc* sc, const Ray* ray) {              /* :272-295 */
    if (sc->skydome) {
        float rcp_pi = 1.0f / PI_32;
        float rcp_2pi = 0.5f / PI_32;
        float phi = atan2f_(ray->d.z, ray->d.x);
        float theta = asinf_(ray->d.y);
        float u = 0.5f + rcp_2pi*phi;
        float v = 0.5f + rcp_pi*theta;
        /* (s32)(u*w) % w with w a u32: the modulo is unsigned */
        uint32_t sx = (uint32_t)(int32_t)(u*(float)sc->skydome_w) % sc->skydome_w;
        uint32_t sy = (uint32_t)(int32_t)(v*(float)sc->skydome_h) % sc->skydome_h;
        return sc->skydome[(size_t)sy*sc->skydome_w + (size_t)sx];
    }
    float st = absf(ray->d.y);
    return lerp3(sc->bot_sky_color, sc->top_sky_color, st);
}

/* a direction from the table: tile k = floor(e n) or its alias, a uniform point of the tile
   (s2), sample_sky's (u, v) mapping inverted */
static V3 env_direction(const EnvTab* t, const rt_scene_desc* sc, float e, V2 s2) {
    float fe = e*(float)t->n;
    uint32_t k = (uint32_t)fe;
    if (k >= t->n) k = t->n - 1;
    float frac = fe - (float)k;
    uint32_t tile = frac < t->prob[k] ? k : t->alias[k];
    uint32_t x0 = (tile % t->tx)*t->tw, y0 = (tile / t->tx)*t->th;
    uint32_t cw = t->tw < sc->skydome_w - x0 ? t->tw : sc->skydome_w - x0;
    uint32_t ch = t->th < sc->skydome_h - y0 ? t->th : sc->skydome_h - y0;
    float u = ((float)x0 + s2.x*(float)cw) / (float)sc->skydome_w;
    float v = ((float)y0 + s2.y*(float)ch) / (float)sc->skydome_h;
    float phi = (u - 0.5f)*(2.0f*PI_32), theta = (v - 0.5f)*PI_32;
    float ct = cosf_(theta);
    return v3(ct*cosf_(phi), sinf_(theta), ct*sinf_(phi));
}

/* sample_sky's texel for d and its tile */
static V3 sky_env(const EnvTab* t, const rt_scene_desc* sc, V3 d, uint32_t* tile) {
    float rcp_pi = 1.0f / PI_32;
    float rcp_2pi = 0.5f / PI_32;
    float u = 0.5f + rcp_2pi*atan2f_(d.z, d.x);
    float v = 0.5f + rcp_pi*asinf_(d.y);
    uint32_t sx = (uint32_t)(int32_t)(u*(float)sc->skydome_w) % sc->skydome_w;
    uint32_t sy = (uint32_t)(int32_t)(v*(float)sc->skydome_h) % sc->skydome_h;
    *tile = (sy / t->th)*t->tx + sx / t->tw;
    return sc->skydome[(size_t)sy*sc->skydome_w + sx];
}

/* solid-angle pdf of env_direction: density / (2 pi^2 cos theta) */
static float env_pdf(const EnvTab* t, uint32_t tile, V3 d) {
    float c2 = 1.0f - d.y*d.y;
    if (!(c2 > 0.0f)) return 0.0f;
    return t->dens[tile] / ((2.0f*PI_32*PI_32)*sqrtf(c2));
}

static inline V3 evaluate_material(const rt_material* m, V3 p) {            /* :297-308 */
    V3 r = m->albedo;
    if (m->flags & RT_MATERIAL_CHECKERS) {
        int32_t ch = (((int32_t)floorf(0.25f*p.x)) ^ ((int32_t)floorf(0.25f*p.z))) & 1;
        if (ch) r = m->checker_color;
    }
    return r;
}

static inline const rt_material* mat_of(const Ctx* ctx, uint32_t id) {
    return id == 0xFFFFu ? ctx->air : &ctx->scene->materials[id];
}

/* advanced_integrator (:581-821) */
static V3 advanced_integrator(Ctx* ctx, Sampler* sampler, RandomSeries* entropy, V3 in_o, V3 in_d) {
    const rt_scene_desc* scene = ctx->scene;
    const rt_settings* st = ctx->settings;
    Ray ray = make_ray(in_o, in_d, FLT_MAX);
    V3 total = v3(0, 0, 0);
    V3 thr = v3(1, 1, 1);
    /* material stack of 64 entries (:601-602); 0xFFFF = the local `air` material */
    int32_t at = 0;
    uint32_t stack[64];
    stack[0] = 0xFFFFu;
    int is_specular = 1;
    V3 prev_N = v3(0, 0, 0);
    for (uint32_t bounce = 0; bounce < st->max_bounce_count; ++bounce) {
        Hit h;
        ctx->closest_rays++;
        intersect_scene_internal(scene, &ray, 0, 0, &h, ctx->ts[0]);
        if (g_gw_on) gpu_walk_query(scene, &ray, 0, 0, ctx->gw[0]);
        V3 N = h.n, I = h.hit_p;
        float t = h.t;
        if (h.hit) {
            float cos_i = -dot(ray.d, N);
            int inside = (cos_i < 0.0f);
            uint32_t surf_id = (h.hit == 1) ? scene->planes[h.index].material_id
                                            : scene->primitives[h.index].material_id;
            const rt_material* surf = &scene->materials[surf_id];
            const rt_material* mi;
            const rt_material* mt;
            if (inside) {
                mi = surf;
                mt = mat_of(ctx, stack[at - 1 > 0 ? at - 1 : 0]);
                cos_i = -cos_i;
                N = neg(N);
            } else {
                mi = mat_of(ctx, stack[at]);
                mt = surf;
            }
            if (mi->is_participating_medium) {                      /* Beer :640-649 */
                V3 ab = v3(expf_(-mi->absorb.x*t), expf_(-mi->absorb.y*t), expf_(-mi->absorb.z*t));
                thr = mul(thr, ab);
            }
            if (mt->flags & RT_MATERIAL_EMISSIVE) {                 /* :651-670 */
                int allow = (!st->next_event_estimation ||
                             ((st->caustics || (bounce < 2)) && is_specular));
                if (allow) {
                    total = add(total, mul(thr, mt->emission_color));
                } else if (bounce > 0 && st->use_mis) {
                    /* the reference looks up light_material but multiplies material_t's
                       emission (RT/integrators.cpp:661-668) */
                    float ldsq = t*t;
                    float light_pdf = ldsq / cos_i;
                    float brdf_pdf = (st->importance_sample_diffuse ? dot(prev_N, ray.d) / PI_32
                                                                    : 1.0f / (2.0f*PI_32));
                    float mis_pdf = light_pdf + brdf_pdf;
                    total = add(total, mul(smul(1.0f / mis_pdf, thr), mt->emission_color));
                }
                break;
            } else {
                float eta_i = mi->ior, eta_t = mt->ior;
                float eta = eta_i / eta_t;
                float cos_t;
                float refl = fresnel_dielectric(cos_i, eta_i, eta_t, eta, &cos_t);
                float reflect_test = get_next_sample_1d(sampler, Sample_Reflectance, bounce);
                refl = lerpf_(refl, 1.0f, mt->metallic);
                is_specular = 1;
                if (reflect_test < refl) {                           /* reflect :684-696 */
                    V3 rd = reflect(ray.d, N);
                    if (mt->roughness > 0.0f) {
                        V3 rs = random_in_unit_sphere(entropy);
                        rd = normalize(add(smul(1.0f + EPSILON, rd), smul(mt->roughness, rs)));
                    }
                    ray = make_ray(add(I, smul(EPSILON, rd)), rd, FLT_MAX);
                    thr = mul(thr, lerp3(v3s(1.0f), mt->albedo, mt->metallic));
                } else {
                    if (mt->is_participating_medium) {               /* refract :698-717 */
                        if (inside) {
                            if (at > 0) --at;
                        } else {
                            if (at < 63) {
                                ++at;
                                stack[at] = (mt == ctx->air) ? 0xFFFFu : (uint32_t)(mt - scene->materials);
                            }
                        }
                        V3 fd = refract(ray.d, N, cos_i, cos_t, eta);
                        ray = make_ray(add(I, muls(fd, EPSILON)), fd, FLT_MAX);
                    } else {                                          /* diffuse :718-790 */
                        is_specular = 0;
                        V3 albedo = evaluate_material(mt, I);
                        V3 brdf = smul(1.0f / PI_32, albedo);
                        const int env = ctx->env != NULL;
                        if (st->next_event_estimation && (scene->light_count > 0 || env)) {
                            float lps = get_next_sample_1d(sampler, Sample_LightSelection, bounce);
                            /* env: the environment is picked with probability q (1 without lights) */
                            const float q = scene->light_count > 0 ? 0.5f : 1.0f;
                            const int pick_env = env && lps < q;
                            if (env) lps = pick_env ? lps / q : (lps - q) / (1.0f - q);
                            float lrp = 0.0f;
                            uint32_t lid = pick_env ? 0u : pick_random_light(ctx, lps, I, &lrp);
                            if (env) lrp = lrp*(1.0f - q);
                            V2 s2 = get_next_sample_2d(sampler, Sample_DirectLighting, bounce);
                            if (pick_env) {
                                V3 L = env_direction(ctx->env, scene, lps, s2);
                                float ndl = dot(N, L);
                                if (ndl > 0.0f) {
                                    uint32_t tile;
                                    V3 Le = sky_env(ctx->env, scene, L, &tile);
                                    float pe = env_pdf(ctx->env, tile, L);
                                    if (pe > 0.0f) {
                                        Hit sh;
                                        Ray sray = make_ray(add(I, muls(L, EPSILON)), L, FLT_MAX);
                                        ctx->shadow_rays++;
                                        if (g_gw_on) gpu_walk_query(scene, &sray, 1, 0, ctx->gw[1]);
                                        if (!intersect_scene_internal(scene, &sray, 1, 0, &sh, ctx->ts[1])) {
                                            float bpdf = (st->importance_sample_diffuse ? ndl / PI_32
                                                                                        : 1.0f / (2.0f*PI_32));
                                            float pdf = st->use_mis ? q*pe + bpdf : q*pe;
                                            total = add(total, mul(mul(muls(thr, ndl / pdf), brdf), Le));
                                        }
                                    }
                                }
                            } else {
                                const rt_primitive* light = &scene->primitives[lid];
                                const rt_material* lmat = &scene->materials[light->material_id];
                                LightSample ls = random_point_on_light(ctx, light, s2, I);
                                V3 L = ls.L, Nl = ls.Nl;
                                float ndl = dot(N, L);
                                float nndl = -dot(Nl, L);
                                if (ndl > 0.0f && nndl > 0.0f) {
                                    Hit sh;
                                    Ray sray = make_ray(add(I, muls(L, EPSILON)), L, ls.dist - 2*EPSILON);
                                    ctx->shadow_rays++;
                                    if (g_gw_on) gpu_walk_query(scene, &sray, 1, lid, ctx->gw[1]);
                                    if (!intersect_scene_internal(scene, &sray, 1, lid, &sh, ctx->ts[1])) {
                                        float sa = (nndl * ls.A) / ls.dist_sq;
                                        float pdf;
                                        if (st->use_mis) {
                                            float lpdf = 1.0f / sa;
                                            float bpdf = (st->importance_sample_diffuse ? ndl / PI_32
                                                                                        : 1.0f / (2.0f*PI_32));
                                            pdf = lpdf + bpdf;
                                        } else {
                                            pdf = 1.0f / sa;
                                        }
                                        pdf *= lrp;
                                        V3 contrib = mul(mul(muls(thr, dot(N, ls.L) / pdf), brdf), lmat->emission_color);
                                        total = add(total, contrib);
                                    }
                                }
                            }
                        }
                        V2 s2 = get_next_sample_2d(sampler, Sample_IndirectLighting, bounce);
                        V3 R;
                        if (st->importance_sample_diffuse) {
                            R = map_to_cosine_weighted_hemisphere(N, s2);
                            thr = muls(thr, PI_32);
                        } else {
                            R = map_to_hemisphere(N, s2);
                            thr = muls(thr, 2.0f*PI_32*dot(N, R));
                        }
                        thr = mul(thr, brdf);
                        ray = make_ray(add(I, muls(N, EPSILON)), R, FLT_MAX);
                    }
                }
            }
            if (st->russian_roulette) {                              /* :801-811 */
                if (!is_specular) {
                    float p = clampf_(max3(thr), 0.1f, 0.9f);
                    float e = get_next_sample_1d(sampler, Sample_Roulette, bounce);
                    if (e > p) break;
                    thr = muls(thr, 1.0f / p);
                }
            }
        } else {
            if (ctx->env) {
                /* leaving a diffuse vertex, which sampled the environment in its NEE: balance
                   heuristic against that pdf; without MIS the NEE alone carries it */
                uint32_t tile;
                V3 Le = sky_env(ctx->env, scene, ray.d, &tile);
                if (!is_specular) {
                    float wgt = 0.0f;
                    if (st->use_mis) {
                        const float q = scene->light_count > 0 ? 0.5f : 1.0f;
                        float pe = env_pdf(ctx->env, tile, ray.d);
                        float bpdf = (st->importance_sample_diffuse ? dot(prev_N, ray.d) / PI_32
                                                                    : 1.0f / (2.0f*PI_32));
                        float den = q*pe + bpdf;
                        wgt = den > 0.0f ? bpdf / den : 0.0f;
                    }
                    Le = smul(wgt, Le);
                }
                total = add(total, mul(thr, Le));
            } else {
                total = add(total, mul(thr, sample_sky(scene, &ray)));
            }
            break;
        }
        prev_N = N;
    }
    return total;
}

/* ====================================================================== */
/* Camera (RT/raytracer.cpp:86-123, 366-475)                               */
/* ====================================================================== */

static V2 transform_bokeh_sample(V2 o, float f, float n, float phi_shutter_max) {    /* :86-94 */
    V2 ab = { (o.x*2.0f) - 1.0f, (o.y*2.0f) - 1.0f };
    V2 phir;
    if ((ab.x*ab.x) > (ab.y*ab.y)) {
        phir.x = (absf(ab.x) > 1e-8f) ? ((PI_32*0.25f)*(ab.y / ab.x)) : 0.0f;
        phir.y = ab.x;
    } else {
        phir.x = (absf(ab.y) > 1e-8f) ? ((PI_32*0.5f) - ((PI_32*0.25f)*(ab.x / ab.y))) : 0.0f;
        phir.y = ab.y;
    }
    phir.x += f*phi_shutter_max;
    if (f > 0.0f) {
        float k = floorf(((n*phir.x) + PI_32) / (2.0f*PI_32));
        phir.y *= powf_(cosf_(PI_32 / n) / cosf_(phir.x - ((2.0f*(PI_32 / n))*k)), f);
    } else {
        phir.y *= 1.0f;
    }
    V2 r = { cosf_(phir.x)*phir.y, sinf_(phir.x)*phir.y };
    return r;
}

static V2 brown_conrady(V2 uv, float amount, float woh) {                    /* :96-107 */
    uv.y /= woh;
    float bd1 = 0.1f*amount, bd2 = -0.025f*amount;
    float r2 = uv.x*uv.x + uv.y*uv.y;
    float fx = 1.0f + r2*bd1 + r2*r2*bd2;
    float fy = 1.0f + r2*bd1 + r2*r2*bd2;
    uv.x *= fx; uv.y *= fy;
    uv.y *= woh;
    return uv;
}

static void apply_lens_distortion(float amount, uint32_t w, uint32_t h, float* u, float* v) {  /* :109-123 */
    float woh = (float)w / (float)h;
    V2 z = {0, 0}, one = {1, 1};
    V2 mn_ = brown_conrady(z, amount, woh);
    V2 mx_ = brown_conrady(one, amount, woh);
    V2 uv = { *u, *v };
    uv = brown_conrady(uv, amount, woh);
    if (amount > 0.0f) {
        uv.x = (uv.x - mn_.x) / (mn_.x + mx_.x);
        uv.y = (uv.y - mn_.y) / (mn_.y + mx_.y);
    }
    *u = uv.x; *v = uv.y;
}

typedef struct {
    V3 cp, cx, cy, cz, film_center;
    float hfw, hfh, pixel_w, pixel_h, lens_radius;
} CamSetup;

static CamSetup cam_setup(const rt_camera* cam, uint32_t w, uint32_t h) {     /* :381-401 */
    CamSetup c;
    c.cp = cam->p; c.cx = cam->x; c.cy = cam->y; c.cz = cam->z;
    float fd = cam->focus_distance;
    c.lens_radius = cam->lens_radius;
    c.hfw = cam->half_film_w * fd;
    c.hfh = cam->half_film_h * fd;
    float film_distance = fd*cam->film_distance;
    c.film_center = sub(c.cp, smul(film_distance, c.cz));
    c.pixel_w = 1.0f / (float)w;
    c.pixel_h = 1.0f / (float)h;
    return c;
}

/* One camera sample of render_tile (:443-474): returns vignetted radiance and jitter. */
static V3 render_sample(Ctx* ctx, const CamSetup* c, RandomSeries* entropy, uint32_t x, uint32_t y,
                        float u, float v, uint32_t canonical, float* jx_out, float* jy_out) {
    const rt_settings* st = ctx->settings;
    Sampler s = { entropy, st->sampling_strategy, canonical, x, y };
    V2 aa = get_next_sample_2d(&s, Sample_AA, 0);
    float jx = aa.x - 0.5f, jy = aa.y - 0.5f;
    V2 dof = get_next_sample_2d(&s, Sample_DOF, 0);
    dof = transform_bokeh_sample(dof, st->f_factor, st->diaphragm_edges, PI_32*st->phi_shutter_max);
    float djx = c->hfw*c->pixel_w*c->lens_radius*dof.x;
    float djy = c->hfh*c->pixel_h*c->lens_radius*dof.y;
    V3 film_p = c->film_center;
    film_p = add(film_p, smul((u + c->pixel_w*jx)*c->hfw, c->cx));
    film_p = add(film_p, smul((v + c->pixel_h*jy)*c->hfh, c->cy));
    V3 jcp = add(add(c->cp, smul(djx, c->cx)), smul(djy, c->cy));
    V3 ro = jcp;
    V3 rd = normalize(sub(film_p, jcp));
    V3 result = advanced_integrator(ctx, &s, entropy, ro, rd);
    float vig = dot(rd, c->cz);
    vig = vig*vig*vig*vig;
    vig = lerpf_(1.0f, vig, st->vignette_strength);
    result = muls(result, vig);
    *jx_out = jx; *jy_out = jy;
    return result;
}

/* splat_filter (:187-259) into a window buffer [win_x0, win_x0+win_w) x [win_y0, ...) of
 * an image of size w x h (window coordinates clip to the image like the reference). */
static void splat(const rt_filter_cache* fc, float* win, int64_t win_x0, int64_t win_y0, int64_t win_w,
                  int64_t w, int64_t h, int64_t x, int64_t y, float jx, float jy, V3 sample) {
    int64_t ks = fc->kernel_size;
    float kscale = (float)(fc->cache_size - 1) / (float)ks;
    float lx[64], ly[64];
    int64_t span = 2*ks + 1;
    for (int64_t i = 0; i < span; ++i) {
        int32_t j = (int32_t)absf(0.5f + kscale*((float)(i - ks) - jx));
        lx[i] = fc->cache[j];
    }
    for (int64_t i = 0; i < span; ++i) {
        int32_t j = (int32_t)absf(0.5f + kscale*((float)(i - ks) - jy));
        ly[i] = fc->cache[j];
    }
    int64_t xm = 0, ym = 0;
    int64_t x0 = x - ks, x1 = x + ks + 1, y0 = y - ks, y1 = y + ks + 1;
    if (x0 < 0) { xm = -x0; x0 = 0; }
    if (y0 < 0) { ym = -y0; y0 = 0; }
    if (x1 > w) x1 = w;
    if (y1 > h) y1 = h;
    for (int64_t sy = y0; sy < y1; ++sy) {
        float fy = ly[ym + (sy - y0)];
        float* row = win + 4*((sy - win_y0)*win_w + (x0 - win_x0));
        for (int64_t sx = x0; sx < x1; ++sx) {
            float fx = lx[xm + (sx - x0)];
            float f = fx*fy;
            row[0] += f*sample.x;
            row[1] += f*sample.y;
            row[2] += f*sample.z;
            row[3] += f;
            row += 4;
        }
    }
}

/* ====================================================================== */
/* Tile renderer + work queue (RT/raytracer.cpp:366-495, 551-603)          */
/* ====================================================================== */

typedef struct {
    const rt_scene_desc* scene;
    const rt_camera* camera;
    const rt_settings* settings;
    const rt_filter_cache* filter;
    uint32_t w, h, tile_w, tile_h, tcx, frame_count, total_frame_index;
    int rng_mode;
    const uint32_t* tiles;        /* tiles to render, in processing order */
    uint32_t tile_count;
    float* direct;                /* non-NULL: splat straight into the frame */
    float** tile_bufs;            /* per listed tile window buffers (threads > 1) */
    atomic_uint next;
    atomic_ullong closest, shadow;
    atomic_ullong ts[2][TS_N];
    rt_material air;
    const EnvTab* env;
} Job;

static void tile_window(const Job* J, uint32_t tile, int64_t* wx0, int64_t* wy0, int64_t* ww, int64_t* wh) {
    int64_t ks = J->filter->cache_size ? J->filter->kernel_size : 0;
    uint32_t min_x = J->tile_w*(tile % J->tcx), min_y = J->tile_h*(tile / J->tcx);
    uint32_t max_x = min_x + J->tile_w < J->w ? min_x + J->tile_w : J->w;
    uint32_t max_y = min_y + J->tile_h < J->h ? min_y + J->tile_h : J->h;
    int64_t x0 = (int64_t)min_x - ks, y0 = (int64_t)min_y - ks;
    int64_t x1 = (int64_t)max_x + ks, y1 = (int64_t)max_y + ks;
    if (x0 < 0) x0 = 0;
    if (y0 < 0) y0 = 0;
    if (x1 > J->w) x1 = J->w;
    if (y1 > J->h) y1 = J->h;
    *wx0 = x0; *wy0 = y0; *ww = x1 - x0; *wh = y1 - y0;
}

static void render_tile(Job* J, uint32_t tile, float* win, int64_t wx0, int64_t wy0, int64_t ww) {
    Ctx ctx;
    memset(&ctx, 0, sizeof(ctx));
    ctx.scene = J->scene; ctx.settings = J->settings; ctx.air = &J->air; ctx.env = J->env;
    const rt_settings* st = J->settings;
    uint32_t min_x = J->tile_w*(tile % J->tcx), min_y = J->tile_h*(tile / J->tcx);
    uint32_t max_x = min_x + J->tile_w < J->w ? min_x + J->tile_w : J->w;
    uint32_t max_y = min_y + J->tile_h < J->h ? min_y + J->tile_h : J->h;
    CamSetup c = cam_setup(J->camera, J->w, J->h);
    uint32_t tile_seed = hash_coordinate3(J->total_frame_index, J->frame_count, tile);
    RandomSeries tile_entropy = random_seed(tile_seed);
    for (uint32_t y = min_y; y < max_y; ++y) {
        float v_ = 1.0f - 2.0f*(float)y*c.pixel_h;
        for (uint32_t x = min_x; x < max_x; ++x) {
            float u_ = 1.0f - 2.0f*(float)x*c.pixel_w;
            float u = u_, v = v_;
            apply_lens_distortion(st->lens_distortion, J->w, J->h, &u, &v);
            for (uint32_t s = 0; s < st->samples_per_pixel; ++s) {
                uint32_t canonical = J->frame_count + s;
                RandomSeries sample_entropy;
                RandomSeries* e = &tile_entropy;
                if (J->rng_mode == RT_RNG_PER_SAMPLE) {
                    sample_entropy = random_seed(oracle_sample_seed(J->total_frame_index, J->frame_count, tile,
                                                                    y*J->w + x, canonical));
                    e = &sample_entropy;
                }
                float jx, jy;
                V3 r = render_sample(&ctx, &c, e, x, y, u, v, canonical, &jx, &jy);
                if (J->filter->cache_size) {
                    splat(J->filter, win, wx0, wy0, ww, J->w, J->h, x, y, jx, jy, r);
                } else {
                    float* px = win + 4*(((int64_t)y - wy0)*ww + ((int64_t)x - wx0));
                    px[0] += r.x; px[1] += r.y; px[2] += r.z; px[3] += 1.0f;
                }
            }
        }
    }
    atomic_fetch_add(&J->closest, ctx.closest_rays);
    atomic_fetch_add(&J->shadow, ctx.shadow_rays);
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < TS_N; ++i) atomic_fetch_add(&J->ts[k][i], ctx.ts[k][i]);
    gw_add(ctx.gw);
}

static void* worker(void* arg) {
    Job* J = (Job*)arg;
    for (;;) {
        uint32_t k = atomic_fetch_add(&J->next, 1u);
        if (k >= J->tile_count) break;
        uint32_t tile = J->tiles[k];
        int64_t wx0, wy0, ww, wh;
        tile_window(J, tile, &wx0, &wy0, &ww, &wh);
        if (J->direct) {
            render_tile(J, tile, J->direct, 0, 0, J->w);
        } else {
            float* buf = (float*)calloc((size_t)(ww*wh*4), sizeof(float));
            render_tile(J, tile, buf, wx0, wy0, ww);
            J->tile_bufs[k] = buf;
        }
    }
    return NULL;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9*(double)ts.tv_nsec;
}

static int validate(const rt_scene_desc* scene, const rt_settings* st, const rt_filter_cache* f) {
    if (!scene || !st || !f) return RT_ERROR_INVALID;
    if (st->integrator != RT_INTEGRATOR_ADVANCED) return RT_ERROR_INVALID;
    if (st->max_bounce_count > 63) return RT_ERROR_INVALID;
    if (f->cache_size && (f->kernel_size == 0 || f->kernel_size > 20 || f->cache_size > 256)) return RT_ERROR_INVALID;
    return RT_OK;
}

/* rt_stats::traversal from the reference's counts (the reference's own TraversalStats, per kind) */
static void set_traversal(rt_stats* stats, const uint64_t ts[2][TS_N]) {
    for (int k = 0; k < 2; ++k) {
        stats->traversal[k].mesh_intersection_count = ts[k][TS_CALLS];
        stats->traversal[k].mesh_bvh_traversals = ts[k][TS_BVH];
        stats->traversal[k].mesh_node_traversals = ts[k][TS_NODES];
        stats->traversal[k].mesh_leaf_traversals = ts[k][TS_LEAVES];
        stats->trace_steps[k] = 0;
    }
}

static void init_air(rt_material* air) {        /* `Material air` RT/integrators.cpp:597-599 */
    memset(air, 0, sizeof(*air));
    air->ior = 1.0f;
    air->is_participating_medium = 1;
}

int oracle_render_tiles(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                        const rt_filter_cache* filter, uint32_t tile_w, uint32_t tile_h,
                        uint32_t total_frame_index, int rng_mode, int threads,
                        uint32_t tile_list_count, const uint32_t* tile_list,
                        rt_accumulation_buffer* accum, rt_stats* stats) {
    int err = validate(scene, settings, filter);
    if (err) return err;
    double t0 = now_s();
    Job* J = (Job*)calloc(1, sizeof(Job));
    J->scene = scene; J->camera = camera; J->settings = settings; J->filter = filter;
    J->w = accum->w; J->h = accum->h; J->tile_w = tile_w; J->tile_h = tile_h;
    J->tcx = (accum->w + tile_w - 1) / tile_w;
    J->frame_count = accum->frame_count; J->total_frame_index = total_frame_index;
    J->rng_mode = rng_mode;
    J->tiles = tile_list; J->tile_count = tile_list_count;
    init_air(&J->air);
    EnvTab env;
    const int have_env = g_env_sampling && settings->next_event_estimation && env_tab_build(scene, &env);
    J->env = have_env ? &env : NULL;
    atomic_init(&J->next, 0u);
    atomic_init(&J->closest, 0ull);
    atomic_init(&J->shadow, 0ull);
    for (int k = 0; k < 2; ++k)
        for (int i = 0; i < TS_N; ++i) atomic_init(&J->ts[k][i], 0ull);
    if (threads <= 1) {
        J->direct = accum->pixels;
        worker(J);
    } else {
        J->tile_bufs = (float**)calloc(tile_list_count, sizeof(float*));
        pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t)*(size_t)threads);
        for (int i = 0; i < threads; ++i) pthread_create(&th[i], NULL, worker, J);
        for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
        free(th);
        for (uint32_t k = 0; k < tile_list_count; ++k) {       /* ordered merge */
            int64_t wx0, wy0, ww, wh;
            tile_window(J, tile_list[k], &wx0, &wy0, &ww, &wh);
            float* b = J->tile_bufs[k];
            for (int64_t yy = 0; yy < wh; ++yy) {
                float* dst = accum->pixels + 4*((wy0 + yy)*(int64_t)accum->w + wx0);
                const float* src = b + 4*yy*ww;
                for (int64_t i = 0; i < 4*ww; ++i) dst[i] += src[i];
            }
            free(b);
        }
        free(J->tile_bufs);
    }
    uint64_t samples = 0;
    for (uint32_t k = 0; k < tile_list_count; ++k) {
        int64_t wx0, wy0, ww, wh;
        uint32_t tile = tile_list[k];
        uint32_t min_x = tile_w*(tile % J->tcx), min_y = tile_h*(tile / J->tcx);
        uint32_t max_x = min_x + tile_w < J->w ? min_x + tile_w : J->w;
        uint32_t max_y = min_y + tile_h < J->h ? min_y + tile_h : J->h;
        (void)wx0; (void)wy0; (void)ww; (void)wh;
        samples += (uint64_t)(max_x - min_x)*(max_y - min_y)*settings->samples_per_pixel;
    }
    if (stats) {
        stats->closest_hit_rays = atomic_load(&J->closest);
        stats->shadow_rays = atomic_load(&J->shadow);
        stats->samples = samples;
        stats->iterations = 0;
        stats->seconds = now_s() - t0;
        uint64_t ts[2][TS_N];
        for (int k = 0; k < 2; ++k)
            for (int i = 0; i < TS_N; ++i) ts[k][i] = atomic_load(&J->ts[k][i]);
        set_traversal(stats, ts);
    }
    if (have_env) env_tab_free(&env);
    free(J);
    return RT_OK;
}

int oracle_render(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                  const rt_filter_cache* filter, const rt_tile_set* tiles,
                  uint32_t total_frame_index, int rng_mode, int threads,
                  rt_accumulation_buffer* accum, rt_stats* stats) {
    if (!tiles || !accum || !accum->pixels || tiles->tile_w == 0 || tiles->tile_h == 0 || tiles->shard_count == 0)
        return RT_ERROR_INVALID;
    uint32_t tcx = (accum->w + tiles->tile_w - 1) / tiles->tile_w;
    uint32_t tcy = (accum->h + tiles->tile_h - 1) / tiles->tile_h;
    uint32_t total = tcx*tcy;
    uint32_t* list = (uint32_t*)malloc(sizeof(uint32_t)*(total ? total : 1));
    uint32_t n = 0;
    /* tile_index = atomic_add(&tile_index, -1) returns the NEW value: tiles total-1 .. 0 (:555) */
    for (uint32_t k = total; k-- > 0;) {
        if (k % tiles->shard_count == tiles->shard_index) list[n++] = k;
    }
    int err = oracle_render_tiles(scene, camera, settings, filter, tiles->tile_w, tiles->tile_h,
                                  total_frame_index, rng_mode, threads, n, list, accum, stats);
    free(list);
    return err;
}

int oracle_trace_samples(const rt_scene_desc* scene, const rt_camera* camera, const rt_settings* settings,
                         uint32_t w, uint32_t h, uint32_t tile_w, uint32_t tile_h,
                         uint32_t frame_count, uint32_t total_frame_index,
                         uint32_t count, const uint32_t* pixel_xy, const uint32_t* sample_offset,
                         float* out, rt_stats* stats) {
    rt_filter_cache box;
    memset(&box, 0, sizeof(box));
    int err = validate(scene, settings, &box);
    if (err) return err;
    rt_material air;
    init_air(&air);
    EnvTab env;
    const int have_env = g_env_sampling && settings->next_event_estimation && env_tab_build(scene, &env);
    Ctx ctx;
    memset(&ctx, 0, sizeof(ctx));
    ctx.scene = scene; ctx.settings = settings; ctx.air = &air; ctx.env = have_env ? &env : NULL;
    CamSetup c = cam_setup(camera, w, h);
    uint32_t tcx = (w + tile_w - 1) / tile_w;
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t x = pixel_xy[2*i], y = pixel_xy[2*i + 1];
        uint32_t tile = (y / tile_h)*tcx + (x / tile_w);
        uint32_t canonical = frame_count + sample_offset[i];
        float u = 1.0f - 2.0f*(float)x*c.pixel_w;
        float v = 1.0f - 2.0f*(float)y*c.pixel_h;
        apply_lens_distortion(settings->lens_distortion, w, h, &u, &v);
        RandomSeries e = random_seed(oracle_sample_seed(total_frame_index, frame_count, tile, y*w + x, canonical));
        float jx, jy;
        V3 r = render_sample(&ctx, &c, &e, x, y, u, v, canonical, &jx, &jy);
        out[5*i + 0] = r.x; out[5*i + 1] = r.y; out[5*i + 2] = r.z;
        out[5*i + 3] = jx; out[5*i + 4] = jy;
    }
    if (have_env) env_tab_free(&env);
    if (stats) {
        stats->closest_hit_rays = ctx.closest_rays;
        stats->shadow_rays = ctx.shadow_rays;
        stats->samples = count;
        stats->iterations = 0;
        stats->seconds = 0;
        set_traversal(stats, ctx.ts);
    }
    gw_add(ctx.gw);
    return RT_OK;
}

int oracle_debug_intersect(const rt_scene_desc* scene, uint32_t count, const rt_ray_query* rays,
                           int occlusion, rt_hit_record* out) {
    for (uint32_t i = 0; i < count; ++i) {
        Ray r = make_ray(rays[i].o, rays[i].d, rays[i].max_t);
        Hit h;
        memset(&h, 0, sizeof(h));
        int hit = intersect_scene_internal(scene, &r, occlusion, rays[i].ignored_primitive, &h, NULL);
        rt_hit_record* o = &out[i];
        memset(o, 0, sizeof(*o));
        o->t = h.t;
        if (!hit) o->primitive = RT_HIT_MISS;
        else o->primitive = (h.hit == 1) ? (RT_HIT_PLANE_BIT | h.index) : h.index;
        if (hit && !occlusion) { o->hit_p = h.hit_p; o->n = h.n; }
    }
    return RT_OK;
}

int oracle_ray_intersect_plane(const float* o, const float* d, const float* n, float dist, float* t) {
    Ray r = make_ray(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), FLT_MAX);
    return ray_intersect_plane(&r, v3(n[0], n[1], n[2]), dist, t);
}
int oracle_ray_intersect_sphere(const float* o, const float* d, float rad, float* t) {
    Ray r = make_ray(v3(o[0], o[1], o[2]), v3(d[0], d[1], d[2]), FLT_MAX);
    return ray_intersect_sphere(&r, rad, t);
}

/* ---- reconstruction filters (RT/reconstruction_filters.cpp:8-106) ---- */
static float sinc_(float x) { return sinf(PI_32*x) / (PI_32*x); }
static float lanczos(float x, float a) {
    x = absf(x);
    if (x < 0.0001f) return 1.0f;
    if (x <= a) return sinc_(x)*sinc_(x / a);
    return 0.0f;
}
static float gaussian(float x, float alpha, float radius) {
    float re = (float)exp(-alpha*radius*radius);
    return mx(0.0f, expf(-alpha*x*x) - re);
}
static float mitchell(float x) {
    const float B = 1.0f / 3.0f, C = 1.0f / 3.0f;
    x = absf(x);
    if (x > 1.0f)
        return (((-B - 6*C)*x*x*x + (6*B + 30*C)*x*x + (-12*B - 48*C)*x + (8*B + 24*C))*(1.0f / 6.0f));
    return (((12 - 9*B - 6*C)*x*x*x + (-18 + 12*B + 6*C)*x*x + (6 - 2*B))*(1.0f / 6.0f));
}

int oracle_load_filter(const char* name, rt_filter_cache* out) {             /* :164-185 */
    memset(out, 0, sizeof(*out));
    int kind;
    uint32_t radius;
    if (!strcmp(name, "Box")) return RT_OK;
    else if (!strcmp(name, "Gaussian 3")) { kind = 1; radius = 3; }
    else if (!strcmp(name, "Gaussian 12")) { kind = 2; radius = 12; }
    else if (!strcmp(name, "Mitchell Netravali")) { kind = 3; radius = 2; }
    else if (!strcmp(name, "Lanczos 3")) { kind = 4; radius = 3; }
    else if (!strcmp(name, "Lanczos 4")) { kind = 5; radius = 4; }
    else if (!strcmp(name, "Lanczos 6")) { kind = 6; radius = 6; }
    else if (!strcmp(name, "Lanczos 12")) { kind = 7; radius = 12; }
    else return RT_OK;   /* find_filter returns Box when not found */
    out->kernel_size = radius;
    out->cache_size = 256;
    for (uint32_t i = 0; i < 256; ++i) {
        float x = ((float)radius*(float)i) / (float)(256 - 1);
        float v = 0;
        switch (kind) {
            case 1: v = gaussian(x, 3.0f, 3.0f); break;
            case 2: v = gaussian(x, 0.03f, 12.0f); break;
            case 3: v = mitchell(x); break;
            case 4: v = lanczos(x, 3.0f); break;
            case 5: v = lanczos(x, 4.0f); break;
            case 6: v = lanczos(x, 6.0f); break;
            case 7: v = lanczos(x, 12.0f); break;
        }
        out->cache[i] = v;
    }
    return RT_OK;
}

/* ======================================================================
 * Output pass (RT/raytracer.cpp:2103-2171)
 * ==================================================================== */
extern const unsigned char rt_dither_rgb1_256[8*256*256*3];   /* data/dither_rgb1_256.u8 */

static float post_clamp(float n, float a, float b) { return mx(a, mn(b, n)); }   /* MathLib clamp */

static float sigmoidal_contrast(float x, float contrast, float midpoint) {      /* RT/raytracer.cpp:69-84 */
    float curve;
    if (x < midpoint) {
        float scale = (1.0f / midpoint)*x;
        curve = midpoint*(scale*scale);
    } else {
        float y = (1.0f / (1.0f - midpoint));
        float scale = y - y*x;
        curve = 1.0f - (1.0f - midpoint)*(scale*scale);
    }
    return x*(1.0f - contrast) + curve*contrast;                                /* lerp(x, curve, contrast) */
}

static float remap_tpdf(float x) {                                              /* RT/raytracer.cpp:125-132 */
    float orig = 2.0f*x - 1.0f;
    x = orig*(1.0f / sqrtf(fabsf(orig)));       /* fast_approx_inverse_square_root = rsqrtss there */
    x = mx(-1.0f, x);
    x = x - (x < 0.0f ? -1.0f : 1.0f);          /* sign_of */
    return x;
}

void oracle_postprocess(const rt_accumulation_buffer* a, const rt_post_settings* post,
                        uint32_t total_frame_index, uint32_t* out) {
    const unsigned char* noise = rt_dither_rgb1_256 + (size_t)(total_frame_index % 8u)*256*256*3;
    size_t i = 0;
    for (uint32_t y = 0; y < a->h; ++y)
        for (uint32_t x = 0; x < a->w; ++x, ++i) {
            const float* s = a->pixels + 4*i;
            float c[3] = {0.0f, 0.0f, 0.0f};
            if ((s[0] != s[0]) || (s[1] != s[1]) || (s[2] != s[2]) || (s[3] != s[3])) {
                c[0] = 0.0f; c[1] = 255.0f; c[2] = 255.0f;
            } else if (s[3] > 0.001f) {
                for (int k = 0; k < 3; ++k) { c[k] = s[k] / s[3]; c[k] = mx(c[k], 0.0f); }
                if (post->exposure != 0.0f) {
                    const float e = powf_(2.0f, post->exposure);
                    for (int k = 0; k < 3; ++k) c[k] = c[k]*e;
                }
                if (post->tonemapping) for (int k = 0; k < 3; ++k) c[k] = 1.0f - expf_(-c[k]);
                if (post->srgb_transform) for (int k = 0; k < 3; ++k) c[k] = powf_(c[k], 1.0f / 2.23333f);
                if (post->contrast != 0.0f)
                    for (int k = 0; k < 3; ++k) c[k] = sigmoidal_contrast(c[k], post->contrast, post->midpoint);
                for (int k = 0; k < 3; ++k) c[k] = c[k]*255.0f;
                const unsigned char* d = noise + 3*((size_t)(y & 255u)*256 + (x & 255u));
                for (int k = 0; k < 3; ++k) c[k] = c[k] + (0.5f + remap_tpdf((1.0f / 255.0f)*(float)d[k]));
            } else if (s[3] < -0.01f) {
                c[0] = -255.0f*s[3]; c[1] = 0.0f; c[2] = -255.0f*s[3];
            }
            uint32_t r = (uint8_t)post_clamp(c[0], 0.0f, 255.0f);
            uint32_t g = (uint8_t)post_clamp(c[1], 0.0f, 255.0f);
            uint32_t b = (uint8_t)post_clamp(c[2], 0.0f, 255.0f);
            out[i] = (255u << 24) | (r << 16) | (g << 8) | b;
        }
}
