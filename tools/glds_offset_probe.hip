// Probe: where does global_load_lds_dwordx4 with an instruction offset land in LDS, and which
// global bytes does it read?  One wave; prints the first float of each 1 KB LDS block.
// hipcc --offload-arch=gfx950 -O3 tools/glds_offset_probe.hip -o tools/glds_offset_probe
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void probe(const float* src, float* out) {
    __shared__ __attribute__((aligned(16))) float lds[2048];
    for (int i = threadIdx.x; i < 2048; i += 64) lds[i] = -1.f;
    __syncthreads();
    const unsigned base = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
    const float* p = src + threadIdx.x * 4;
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off offset:1024\n\t"
        "s_mov_b32 m0, %0\n\ts_waitcnt vmcnt(0)"
        : "=&s"(keep)
        : "v"(p), "s"(__builtin_amdgcn_readfirstlane(base))
        : "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 2048; i += 64) out[i] = lds[i];
}

int main() {
    float h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (float)i;
    float *src, *out;
    (void)hipMalloc(&src, sizeof(h));
    (void)hipMalloc(&out, 2048 * 4);
    (void)hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, src, out);
    float o[2048];
    (void)hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
    for (int b = 0; b < 8; ++b) printf("lds block %d (byte %d): first float %.0f, last float %.0f\n", b, b * 1024, o[b * 256], o[b * 256 + 255]);
    return 0;
}
