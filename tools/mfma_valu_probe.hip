// Micro-probe: cycles per v_mfma_f32_32x32x16_bf16 in a single-accumulator chain with N VALU
// fillers after each MFMA (one wave per SIMD, 256 blocks x 4 waves), for the filler kinds the step
// kernel's epilogues use.  hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_probe.hip -o /tmp/probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KIND, int N>
__global__ __launch_bounds__(256) void probe(float* out, unsigned long long* cyc, int iters) {
    f32x16 acc = {};
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = (__bf16)(0.001f * (threadIdx.x + i));
        b[i] = (__bf16)(0.002f * (threadIdx.x - i));
    }
    float x[12];
    uint32_t bits = 0;
    for (int i = 0; i < 12; ++i) x[i] = threadIdx.x * 0.5f + i;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            __builtin_amdgcn_sched_barrier(0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            if constexpr (KIND == 0) {  // independent v_add_f32
#pragma unroll
                for (int j = 0; j < N; ++j) asm volatile("v_add_f32_e32 %0, 1.0, %0" : "+v"(x[j]));
            } else if constexpr (KIND == 1) {  // the VCC relu + mask-bit triple (N/3 of them)
#pragma unroll
                for (int j = 0; j < N / 3; ++j) {
                    float y;
                    asm volatile(
                        "v_cmp_lt_f32_e32 vcc, 0, %2\n\t"
                        "v_cndmask_b32_e32 %0, 0, %2, vcc\n\t"
                        "v_addc_co_u32_e32 %1, vcc, %1, %1, vcc"
                        : "=&v"(y), "+v"(bits)
                        : "v"(x[j])
                        : "vcc");
                    x[j + 1] += y;
                }
            } else if constexpr (KIND == 2) {  // reading the accumulator (v_accvgpr_read) + add
#pragma unroll
                for (int j = 0; j < N; ++j) x[j] += acc[j];
            } else {  // the bf16 hi / lo packing block (6 VALU)
#pragma unroll
                for (int j = 0; j < N / 6; ++j) {
                    uint32_t w, wl, t0_, t1_;
                    asm volatile(
                        "v_cvt_pk_bf16_f32 %0, %4, %5\n\t"
                        "v_lshlrev_b32_e32 %2, 16, %0\n\t"
                        "v_and_b32_e32 %3, 0xffff0000, %0\n\t"
                        "v_sub_f32_e32 %2, %4, %2\n\t"
                        "v_sub_f32_e32 %3, %5, %3\n\t"
                        "v_cvt_pk_bf16_f32 %1, %2, %3"
                        : "=&v"(w), "=&v"(wl), "=&v"(t0_), "=&v"(t1_)
                        : "v"(x[2 * j]), "v"(x[2 * j + 1]));
                    x[2 * j] = __uint_as_float(w);
                    x[2 * j + 1] = __uint_as_float(wl);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int i = 0; i < 16; ++i) s += acc[i];
    for (int i = 0; i < 12; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s + bits;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int N>
void run(const char* name, float* out, unsigned long long* cyc) {
    const int iters = 200;
    hipLaunchKernelGGL((probe<KIND, N>), dim3(256), dim3(256), 0, 0, out, cyc, iters);
    hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < 256; ++i) m += (double)h[i];
    m /= 256.0;
    printf("%-28s N=%2d  %.1f cycles per MFMA\n", name, N, m / (iters * 16.0));
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 256 * 4);
    hipMalloc(&cyc, 256 * 8);
    run<0, 0>("bare chain", out, cyc);
    run<0, 3>("v_add_f32", out, cyc);
    run<0, 5>("v_add_f32", out, cyc);
    run<0, 8>("v_add_f32", out, cyc);
    run<1, 3>("relu+mask (VCC)", out, cyc);
    run<1, 6>("relu+mask (VCC)", out, cyc);
    run<2, 1>("accvgpr read + add", out, cyc);
    run<2, 2>("accvgpr read + add", out, cyc);
    run<3, 6>("bf16 hi/lo pack", out, cyc);
    return 0;
}
