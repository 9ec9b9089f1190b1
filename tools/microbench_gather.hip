// Microbenchmark: how a wave fetches 64 random 128-byte lines (one BVH4 node per lane, the trace
// kernels' step).  A: each lane loads its own line as 8 x 16-byte loads (the current step: every
// wave-instruction touches 64 lines).  B: the wave loads the 64 lines cooperatively (8 lanes per
// line, every wave-instruction touches 8 whole lines) and hands them out through LDS.  C: B with
// the loads written straight into LDS (global_load_lds_dwordx4).  Each lane's next line depends on
// the data of its current one (a dependent chain, as in traversal).
//   hipcc --offload-arch=gfx950 -O3 -o mbg tools/microbench_gather.hip && ./mbg
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}
__device__ __forceinline__ uint32_t fold(const uint4 (&v)[8]) {
    uint32_t a = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) a ^= v[k].x + v[k].y * 3u + v[k].z * 5u + v[k].w * 7u;
    return a;
}

__global__ void __launch_bounds__(256) gather_lane(const uint4* buf, uint32_t mask, int steps, uint32_t* out) {
    const uint32_t g = blockIdx.x*blockDim.x + threadIdx.x;
    uint32_t idx = hash(g) & mask, acc = 0;
    for (int s = 0; s < steps; ++s) {
        const uint4* p = buf + 8*(size_t)idx;
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[k];
        const uint32_t f = fold(v);
        acc += f;
        idx = (f ^ hash(idx + s)) & mask;
    }
    out[g] = acc;
}

__global__ void __launch_bounds__(256) gather_coop(const uint4* buf, uint32_t mask, int steps, uint32_t* out) {
    __shared__ uint4 stage[4][512];                 // 8 KB per wave
    const uint32_t g = blockIdx.x*blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t idx = hash(g) & mask, acc = 0;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t li = __shfl(idx, 8*i + (lane >> 3));
            stage[w][i*64 + lane] = buf[8*(size_t)li + (lane & 7u)];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint4 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = stage[w][(lane >> 3)*64 + 8*(lane & 7u) + m];
        const uint32_t f = fold(v);
        acc += f;
        idx = (f ^ hash(idx + s)) & mask;
        __builtin_amdgcn_wave_barrier();
    }
    out[g] = acc;
}

__global__ void __launch_bounds__(256) gather_coop_lds(const uint4* buf, uint32_t mask, int steps, uint32_t* out) {
    __shared__ uint4 stage[4][512];
    const uint32_t g = blockIdx.x*blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t idx = hash(g) & mask, acc = 0;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t li = __shfl(idx, 8*i + (lane >> 3));
            __builtin_amdgcn_global_load_lds(buf + 8*(size_t)li + (lane & 7u), &stage[w][i*64], 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0);              // vmcnt(0) lgkmcnt(0): the DMA has landed
        __builtin_amdgcn_wave_barrier();
        uint4 v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = stage[w][(lane >> 3)*64 + 8*(lane & 7u) + m];
        const uint32_t f = fold(v);
        acc += f;
        idx = (f ^ hash(idx + s)) & mask;
        __builtin_amdgcn_wave_barrier();
    }
    out[g] = acc;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int steps = 256;
    const uint32_t max_lines = 1u << 20;             // 128 MB
    std::vector<uint32_t> h(max_lines*32);
    uint32_t x = 12345;
    for (auto& e : h) { x = x*1664525u + 1013904223u; e = x; }
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, (size_t)max_lines*128));
    CK(hipMemcpy(buf, h.data(), (size_t)max_lines*128, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, (size_t)cus*16*256*4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    printf("cus %d, steps %d; ns per lane-step and lines per ns chip-wide\n", cus, steps);
    for (uint32_t lines : {1u << 14, 1u << 18, 1u << 20}) {
        for (int bpc : {1, 2, 3, 4}) {                // 256-thread blocks per CU: 4, 8, 12, 16 waves per CU
            const int grid = cus*bpc;
            for (int kind = 0; kind < 3; ++kind) {
                auto launch = [&]() {
                    if (kind == 0) gather_lane<<<grid, 256>>>(buf, lines - 1, steps, out);
                    else if (kind == 1) gather_coop<<<grid, 256>>>(buf, lines - 1, steps, out);
                    else gather_coop_lds<<<grid, 256>>>(buf, lines - 1, steps, out);
                };
                launch();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a));
                for (int r = 0; r < 3; ++r) launch();
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                const double lane_steps = 3.0*grid*256.0*steps;
                printf("lines %7u (%6.1f MB) waves/CU %2d %-10s %8.3f ms  %7.2f ns/lane-step  %6.2f lines/ns\n", lines,
                       lines*128.0/1e6, bpc*4, kind == 0 ? "per-lane" : kind == 1 ? "coop" : "coop-lds", ms,
                       ms*1e6/(lane_steps/(grid*256.0)), lane_steps/(ms*1e6));
            }
        }
    }
    return 0;
}
