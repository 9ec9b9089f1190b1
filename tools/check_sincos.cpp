// Host check that d_sincosf(x) gives exactly d_sinf(x) and d_cosf(x), bit for bit, for every float
// (the device math is plain IEEE f32 without contraction, so the host build computes the same bits).
//   g++ -O2 -ffp-contract=off -DRT_DMATH_HOST_TEST -DRT_RCP_CR=0 -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
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
int main() {
    unsigned long long bad = 0;
    for (uint64_t u = 0; u <= 0xFFFFFFFFull; ++u) {
        float x; uint32_t b = (uint32_t)u; memcpy(&x, &b, 4);
        float s, c; d_sincosf(x, s, c);
        const float s1 = d_sinf(x), c1 = d_cosf(x);
        if (memcmp(&s, &s1, 4) || memcmp(&c, &c1, 4)) {
            if (bad < 10) printf("mismatch x=%08x sin %08x/%08x cos %08x/%08x\n", b, *(uint32_t*)&s, *(uint32_t*)&s1,
                                 *(uint32_t*)&c, *(uint32_t*)&c1);
            ++bad;
        }
    }
    printf("%llu mismatches over all 2^32 floats\n", bad);
    return bad ? 1 : 0;
}
