// Host check that d_sincosf(x) gives exactly d_sinf(x) and d_cosf(x), bit for bit, for every float
// (the device math is plain IEEE f32 without contraction, so the host build computes the same bits).
//   g++ -O2 -ffp-contract=off -DRT_DMATH_HOST_TEST -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
//       tools/check_sincos.cpp -o /tmp/check_sincos && /tmp/check_sincos
#include <cstdio>
#include <cstring>
#include <cstdint>
static inline uint32_t __float_as_uint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float __uint_as_float(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline int __float_as_int(float f) { int u; memcpy(&u, &f, 4); return u; }
static inline float __int_as_float(int u) { float f; memcpy(&f, &u, 4); return f; }
#include "../buas-pathtracer_amd/csrc/rt_dmath.h"
using namespace rtd;
#include <cstdlib>
// argv[1]: stride through the 2^32 bit patterns (default 1: all of them; tests/test_dmath_sincos.py uses a
// prime stride plus every pattern near the range-reduction boundaries)
int main(int argc, char** argv) {
    const uint64_t stride = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1;
    unsigned long long bad = 0, n = 0;
    auto check = [&](uint32_t b) {
        float x; memcpy(&x, &b, 4);
        float s, c; d_sincosf(x, s, c);
        const float s1 = d_sinf(x), c1 = d_cosf(x);
        ++n;
        if (memcmp(&s, &s1, 4) || memcmp(&c, &c1, 4)) {
            if (bad < 10) printf("mismatch x=%08x sin %08x/%08x cos %08x/%08x\n", b, *(uint32_t*)&s, *(uint32_t*)&s1,
                                 *(uint32_t*)&c, *(uint32_t*)&c1);
            ++bad;
        }
    };
    // every float within 2^16 ulps of +-0, +-8192 (the reduction's limit), +-inf and the octant boundaries k*pi/4
    const float anchors[] = {0.0f, 8192.0f, __builtin_inff(), 0.785398163f, 1.570796327f, 2.35619449f, 3.141592654f,
                             3.926990817f, 4.71238898f, 5.497787144f, 6.283185307f};
    for (float a : anchors)
        for (int sg = 0; sg < 2; ++sg) {
            uint32_t b; const float v = sg ? -a : a; memcpy(&b, &v, 4);
            for (int64_t d = -65536; d <= 65536; ++d) check((uint32_t)((int64_t)b + d));
        }
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; u += stride) check((uint32_t)u);
    printf("%llu mismatches over %llu floats\n", bad, n);
    return bad ? 1 : 0;
}
