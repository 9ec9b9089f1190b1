#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(const float* g, float* out) {
    __shared__ float st[64*4 + 64];
    for (int i = threadIdx.x; i < 64*4 + 64; i += 64) st[i] = -1.0f;
    __syncthreads();
    __builtin_amdgcn_global_load_lds(g + 3*threadIdx.x, &st[0], 12, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64*4 + 64; i += 64) out[i] = st[i];
}
int main() {
    float h[192]; for (int i = 0; i < 192; ++i) h[i] = (float)i;
    float *g, *o; hipMalloc(&g, sizeof h); hipMalloc(&o, 320*4);
    hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
    k<<<1, 64>>>(g, o); hipDeviceSynchronize();
    float r[320]; hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    for (int i = 0; i < 320; ++i) printf("%g%c", r[i], (i % 16 == 15) ? '\n' : ' ');
    return 0;
}
