// Microbenchmark: path-state layout for the wavefront loop (DESIGN.md §6 "path pool").
// Models k_shade (every slot: read 8 float4, write 6 float4 for the ~83 % still running) and
// k_generate (a random 25 % of slots: read the 3 float4 a splat needs, write 8 float4 of new
// path state) with the state either SoA (8 arrays of float4, the current pool) or AoS (one
// 128-byte line per slot).  hipcc --offload-arch=gfx950 -O3 -o mb tools/microbench_layout.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
typedef float nt4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 ldn(const float4* p) {
    const nt4 v = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p)); return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stn(float4* p, float4 v) {
    const nt4 t = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(t, reinterpret_cast<nt4*>(p));
}

// shade-like pass
__global__ void shade_soa(float4* const* a, uint32_t n, uint32_t it) {
    const uint32_t i = blockIdx.x*blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ldn(a[k] + i);
    if ((hash(i ^ it) & 1023u) < 850u) {
        float4 s = v[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
#pragma unroll
        for (int k = 0; k < 6; ++k) stn(a[k] + i, make_float4(s.x + k, s.y, s.z, v[k].w));
    }
}
__global__ void shade_aos(float4* a, uint32_t n, uint32_t it) {
    const uint32_t i = blockIdx.x*blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ldn(a + 8*(size_t)i + k);
    if ((hash(i ^ it) & 1023u) < 850u) {
        float4 s = v[0];
#pragma unroll
        for (int k = 1; k < 8; ++k) { s.x += v[k].x; s.y += v[k].y; s.z += v[k].z; s.w += v[k].w; }
#pragma unroll
        for (int k = 0; k < 6; ++k) stn(a + 8*(size_t)i + k, make_float4(s.x + k, s.y, s.z, v[k].w));
    }
}
// generate-like pass: a random quarter of the slots is splatted and re-initialised
__global__ void gen_soa(float4* const* a, float4* rec, uint32_t n, uint32_t it) {
    const uint32_t i = blockIdx.x*blockDim.x + threadIdx.x;
    if (i >= n || (hash(i + 77u*it) & 3u)) return;
    const float4 L = a[3][i], j = a[6][i], d = a[1][i];
    stn(rec + i, make_float4(L.x + j.x, L.y + j.y, L.z, d.w));
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k][i] = make_float4((float)k, (float)i, 1.0f, 0.5f);
}
__global__ void gen_aos(float4* a, float4* rec, uint32_t n, uint32_t it) {
    const uint32_t i = blockIdx.x*blockDim.x + threadIdx.x;
    if (i >= n || (hash(i + 77u*it) & 3u)) return;
    float4* p = a + 8*(size_t)i;
    const float4 L = p[3], j = p[6], d = p[1];
    stn(rec + i, make_float4(L.x + j.x, L.y + j.y, L.z, d.w));
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = make_float4((float)k, (float)i, 1.0f, 0.5f);
}

int main() {
    const uint32_t n = 6291456;                     // one partition's pool (C3)
    std::vector<float4*> soa(8);
    for (auto& p : soa) { CK(hipMalloc(&p, 16ull*n)); CK(hipMemset(p, 0, 16ull*n)); }
    float4** dsoa; CK(hipMalloc(&dsoa, sizeof(float4*)*8)); CK(hipMemcpy(dsoa, soa.data(), sizeof(float4*)*8, hipMemcpyHostToDevice));
    float4* aos; CK(hipMalloc(&aos, 128ull*n)); CK(hipMemset(aos, 0, 128ull*n));
    float4* rec; CK(hipMalloc(&rec, 16ull*n));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const uint32_t B = 256, G = (n + B - 1) / B;
    auto timeit = [&](const char* name, auto launch, double bytes) {
        for (int w = 0; w < 3; ++w) launch(w);
        (void)hipEventRecord(e0);
        const int R = 20;
        for (int r = 0; r < R; ++r) launch(r + 3);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s %8.1f us/launch  %7.1f GB/s of touched bytes\n", name, 1e3*ms/R, bytes / (1e-3*ms/R) / 1e9);
    };
    const double shade_bytes = n*(128.0 + 0.83*96.0), gen_bytes = 0.25*n*(48.0 + 16.0 + 128.0);
    for (int rep = 0; rep < 2; ++rep) {
        timeit("shade_soa", [&](int r) { shade_soa<<<G, B>>>(dsoa, n, r); }, shade_bytes);
        timeit("shade_aos", [&](int r) { shade_aos<<<G, B>>>(aos, n, r); }, shade_bytes);
        timeit("gen_soa", [&](int r) { gen_soa<<<G, B>>>(dsoa, rec, n, r); }, gen_bytes);
        timeit("gen_aos", [&](int r) { gen_aos<<<G, B>>>(aos, rec, n, r); }, gen_bytes);
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}
