// mfma_acc_probe.hip -- accumulation error of v_mfma_f32_32x32x16_bf16 vs v_mfma_f32_16x16x32_bf16
// on the same K = 256 dot products (random bf16 operands, one wave), against exact (fp64) sums and an
// fp32 sequential FMA chain.  Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_acc_probe.hip -o /tmp/probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

constexpr int M = 32, N = 32, K = 256;

// A [M][K], B [K][N] bf16 bits; out32 / out16 [M][N]
__global__ void probe(const u16* A, const u16* B, float* out32, float* out16) {
    const int lane = threadIdx.x;
    {  // 32x32x16: lane l holds A[l & 31][k0 + 8 (l >> 5) + j], B[k0 + 8 (l >> 5) + j][l & 31]
        f32x16 acc = {};
        for (int k0 = 0; k0 < K; k0 += 16) {
            u16 a[8], b[8];
            for (int j = 0; j < 8; ++j) {
                a[j] = A[(lane & 31) * K + k0 + 8 * (lane >> 5) + j];
                b[j] = B[(k0 + 8 * (lane >> 5) + j) * N + (lane & 31)];
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8*>(a), *reinterpret_cast<bf16x8*>(b),
                                                          acc, 0, 0, 0);
        }
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            out32[row * N + (lane & 31)] = acc[r];
        }
    }
    for (int bm = 0; bm < 2; ++bm)
        for (int bn = 0; bn < 2; ++bn) {  // 16x16x32: lane l holds A[l & 15][k0 + 8 (l >> 4) + j]
            f32x4 acc = {};
            for (int k0 = 0; k0 < K; k0 += 32) {
                u16 a[8], b[8];
                for (int j = 0; j < 8; ++j) {
                    a[j] = A[(16 * bm + (lane & 15)) * K + k0 + 8 * (lane >> 4) + j];
                    b[j] = B[(k0 + 8 * (lane >> 4) + j) * N + 16 * bn + (lane & 15)];
                }
                acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(a), *reinterpret_cast<bf16x8*>(b),
                                                              acc, 0, 0, 0);
            }
            for (int r = 0; r < 4; ++r) out16[(16 * bm + 4 * (lane >> 4) + r) * N + 16 * bn + (lane & 15)] = acc[r];
        }
}

static float bf(u16 h) {
    unsigned u = (unsigned)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static u16 tobf(float f) {
    unsigned u;
    std::memcpy(&u, &f, 4);
    u += 0x7fff + ((u >> 16) & 1);
    return (u16)(u >> 16);
}

int main() {
    srand(7);
    std::vector<u16> A(M * K), B(K * N);
    // activations-like (non-negative, ReLU'd) B and signed weights A, several magnitudes
    for (auto& x : A) x = tobf(((float)rand() / RAND_MAX - 0.5f) * 0.2f);
    for (auto& x : B) x = tobf((rand() % 3 == 0) ? 0.f : (float)rand() / RAND_MAX * 2.f);
    u16 *dA, *dB;
    float *d32, *d16;
    hipMalloc(&dA, A.size() * 2);
    hipMalloc(&dB, B.size() * 2);
    hipMalloc(&d32, M * N * 4);
    hipMalloc(&d16, M * N * 4);
    hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(dA, dB, d32, d16);
    std::vector<float> o32(M * N), o16(M * N);
    hipMemcpy(o32.data(), d32, M * N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o16.data(), d16, M * N * 4, hipMemcpyDeviceToHost);
    double e32 = 0, e16 = 0, efma = 0, m32 = 0, m16 = 0, mfma = 0, scale = 0;
    int diff = 0;
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < N; ++j) {
            double ex = 0, aa = 0;
            float ch = 0.f;
            for (int k = 0; k < K; ++k) {
                const double p = (double)bf(A[i * K + k]) * bf(B[k * N + j]);
                ex += p;
                aa += fabs(p);
                ch = fmaf(bf(A[i * K + k]), bf(B[k * N + j]), ch);
            }
            const double r32 = fabs(o32[i * N + j] - ex) / aa, r16 = fabs(o16[i * N + j] - ex) / aa, rf = fabs(ch - ex) / aa;
            e32 += r32;
            e16 += r16;
            efma += rf;
            m32 = fmax(m32, r32);
            m16 = fmax(m16, r16);
            mfma = fmax(mfma, rf);
            scale += aa;
            diff += o32[i * N + j] != o16[i * N + j];
        }
    const int n = M * N;
    printf("error / sum|products| over %d dot products of K=%d:\n", n, K);
    printf("  32x32x16 MFMA chain : mean %.3e  max %.3e\n", e32 / n, m32);
    printf("  16x16x32 MFMA chain : mean %.3e  max %.3e\n", e16 / n, m16);
    printf("  fp32 sequential fma : mean %.3e  max %.3e\n", efma / n, mfma);
    printf("  32x32x16 != 16x16x32 in %d of %d outputs\n", diff, n);
    return 0;
}
