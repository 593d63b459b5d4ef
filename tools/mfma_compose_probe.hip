// mfma_compose_probe.hip -- can k_step3's 16x16x32 MFMAs reproduce k_step2's 32x32x16 accumulation
// sequence bit for bit?  k_step2 accumulates, per 16-k chunk c of a split-bf16 layer,
//   forward: hi.hi(c), hi.lo(c), lo.hi(c)       dgrad: W_hi^T dz(c), W_lo^T dz(c)
// with one v_mfma_f32_32x32x16_bf16 per term.  A 16x16x32 MFMA covers two 16-k halves (lane groups
// 0-1 and 2-3); if the hardware adds the halves in order, these compositions give the same bits:
//   forward pair (2s, 2s+1): [hh(2s) | hl(2s)], [lh(2s) | hh(2s+1)], [hl(2s+1) | lh(2s+1)]
//   dgrad chunk c: [hd(c) | ld(c)]
//   dW_last (k_step2: one K = 32-pixel MFMA from acc 0): pixels 0-15 from acc 0 (other half zero),
//   then pixels 16-31 from that partial (first half zero).
// Random operands shaped like the kernel's (ReLU'd activations with zeros, signed weights split
// into bf16 hi + lo), several magnitude scales; prints the count of differing outputs per test.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mfma_compose_probe.hip -o tools/mfma_compose_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16;

// seq: n MFMAs, fragments [n][64][8] bf16 for A and B; init [64][16] (32x32) or [64][4] (16x16)
__global__ void run32(const u16* A, const u16* B, int n, const float* init, float* out) {
    const int l = threadIdx.x;
    f32x16 acc;
    for (int r = 0; r < 16; ++r) acc[r] = init[l * 16 + r];
    for (int i = 0; i < n; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + ((size_t)i * 64 + l) * 8);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + ((size_t)i * 64 + l) * 8);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 16; ++r) out[l * 16 + r] = acc[r];
}
__global__ void run16(const u16* A, const u16* B, int n, const float* init, float* out) {
    const int l = threadIdx.x;
    f32x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = init[l * 4 + r];
    for (int i = 0; i < n; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + ((size_t)i * 64 + l) * 8);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + ((size_t)i * 64 + l) * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

// as run16, with a per-MFMA B lane-group pattern (blgp 0: as is, 1: lanes 0-31 also into 32-63,
// 2: lanes 32-63 also into 0-31)
__global__ void run16g(const u16* A, const u16* B, const int* g, int n, const float* init, float* out) {
    const int l = threadIdx.x;
    f32x4 acc;
    for (int r = 0; r < 4; ++r) acc[r] = init[l * 4 + r];
    for (int i = 0; i < n; ++i) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + ((size_t)i * 64 + l) * 8);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(B + ((size_t)i * 64 + l) * 8);
        if (g[i] == 1) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 1);
        else if (g[i] == 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 2);
        else acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

static u16 tobf(float f) {
    unsigned u;
    std::memcpy(&u, &f, 4);
    u += 0x7fff + ((u >> 16) & 1);
    return (u16)(u >> 16);
}
static float bf(u16 h) {
    unsigned u = (unsigned)h << 16;
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// logical operands: a "term" is a 16-row x 16-k block of A (rows m, k) and a 16-k x 16-col block of B
struct Blk {
    u16 a[16][16];  // [m][k]
    u16 b[16][16];  // [k][n]
};

// one 32x32x16 MFMA of a term (rows / cols 16..31 zero)
static void frag32(const Blk& t, u16* A, u16* B) {
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
            const int row = l & 31, col = l & 31, k = 8 * (l >> 5) + j;
            A[l * 8 + j] = row < 16 ? t.a[row][k] : 0;
            B[l * 8 + j] = col < 16 ? t.b[k][col] : 0;
        }
}
// one 16x16x32 MFMA of two terms (k 0..15: t0, 16..31: t1); null = zero half
static void frag16(const Blk* t0, const Blk* t1, u16* A, u16* B) {
    for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
            const int row = l & 15, col = l & 15, k = 8 * (l >> 4) + j;
            const Blk* t = k < 16 ? t0 : t1;
            const int kk = k & 15;
            A[l * 8 + j] = t ? t->a[row][kk] : 0;
            B[l * 8 + j] = t ? t->b[kk][col] : 0;
        }
}

struct Runner {
    u16 *dA, *dB;
    float *dI, *dO;
    Runner() {
        hipMalloc(&dA, 512 * 64 * 8 * 2);
        hipMalloc(&dB, 512 * 64 * 8 * 2);
        hipMalloc(&dI, 64 * 16 * 4);
        hipMalloc(&dO, 64 * 16 * 4);
    }
    // result as a [16][16] block (rows m, cols n)
    void go32(const std::vector<Blk>& seq, const float init[16][16], float out[16][16]) {
        const int n = (int)seq.size();
        std::vector<u16> A(n * 512), B(n * 512);
        for (int i = 0; i < n; ++i) frag32(seq[i], &A[i * 512], &B[i * 512]);
        std::vector<float> I(64 * 16, 0.f), O(64 * 16);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
                if (row < 16 && col < 16) I[l * 16 + r] = init[row][col];
            }
        hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dI, I.data(), I.size() * 4, hipMemcpyHostToDevice);
        run32<<<1, 64>>>(dA, dB, n, dI, dO);
        hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 16; ++r) {
                const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
                if (row < 16 && col < 16) out[row][col] = O[l * 16 + r];
            }
    }
    // blgp: per MFMA; the B fragments of seq are built as given, the pattern applied by the hardware
    void go16(const std::vector<std::pair<const Blk*, const Blk*>>& seq, const float init[16][16], float out[16][16],
              const std::vector<std::pair<const Blk*, const Blk*>>* bseq = nullptr, const std::vector<int>* blgp = nullptr) {
        const int n = (int)seq.size();
        std::vector<u16> A(n * 512), B(n * 512), tmp(512);
        for (int i = 0; i < n; ++i) {
            frag16(seq[i].first, seq[i].second, &A[i * 512], &B[i * 512]);
            if (bseq) frag16((*bseq)[i].first, (*bseq)[i].second, tmp.data(), &B[i * 512]);
        }
        std::vector<float> I(64 * 4), O(64 * 4);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) I[l * 4 + r] = init[4 * (l >> 4) + r][l & 15];
        hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
        hipMemcpy(dI, I.data(), I.size() * 4, hipMemcpyHostToDevice);
        if (blgp) {
            int* dg;
            hipMalloc(&dg, n * 4);
            hipMemcpy(dg, blgp->data(), n * 4, hipMemcpyHostToDevice);
            run16g<<<1, 64>>>(dA, dB, dg, n, dI, dO);
            hipDeviceSynchronize();
            hipFree(dg);
        } else {
            run16<<<1, 64>>>(dA, dB, n, dI, dO);
        }
        hipMemcpy(O.data(), dO, O.size() * 4, hipMemcpyDeviceToHost);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r) out[4 * (l >> 4) + r][l & 15] = O[l * 4 + r];
    }
};

static int ndiff(const float x[16][16], const float y[16][16]) {
    int d = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) d += std::memcmp(&x[i][j], &y[i][j], 4) != 0;
    return d;
}

int main() {
    std::mt19937 rng(11);
    std::uniform_real_distribution<float> U(-1.f, 1.f);
    Runner R;
    const int NCH = 16;  // 16-k chunks: K = 256
    long long tot[5] = {0, 0, 0, 0, 0}, outs[5] = {0, 0, 0, 0, 0};
    for (int trial = 0; trial < 48; ++trial) {
        const float ws = std::ldexp(1.f, (int)(rng() % 9) - 6), xs = std::ldexp(1.f, (int)(rng() % 9) - 4);
        // weights W [16][256] (hi + lo), activations X [256][16] (hi + lo, ReLU'd, ~40% zeros), dz [256][16]
        std::vector<float> W(16 * 256), X(256 * 16), D(256 * 16);
        for (auto& v : W) v = U(rng) * ws;
        for (auto& v : X) v = (rng() % 5 < 2) ? 0.f : std::fabs(U(rng)) * xs;
        for (auto& v : D) v = (rng() % 4 == 0) ? 0.f : U(rng) * xs * 1e-3f;
        float bias[16][16];
        for (int i = 0; i < 16; ++i) {
            const float b0 = U(rng) * ws;
            for (int j = 0; j < 16; ++j) bias[i][j] = b0;
        }
        // chunk terms
        std::vector<Blk> hh(NCH), hl(NCH), lh(NCH), hd(NCH), ld(NCH);
        for (int c = 0; c < NCH; ++c)
            for (int m = 0; m < 16; ++m)
                for (int k = 0; k < 16; ++k) {
                    const float w = W[m * 256 + 16 * c + k];
                    const u16 wh = tobf(w), wl = tobf(w - bf(wh));
                    hh[c].a[m][k] = hl[c].a[m][k] = wh;
                    lh[c].a[m][k] = wl;
                    hd[c].a[m][k] = wh;  // (the dgrad's W^T block: any 16x16 weight block will do)
                    ld[c].a[m][k] = wl;
                    for (int n = 0; n < 16; ++n) {
                        const float x = X[(16 * c + k) * 16 + n];
                        const u16 xh = tobf(x), xl = tobf(x - bf(xh));
                        hh[c].b[k][n] = lh[c].b[k][n] = xh;
                        hl[c].b[k][n] = xl;
                        hd[c].b[k][n] = ld[c].b[k][n] = tobf(D[(16 * c + k) * 16 + n]);
                    }
                }
        float r2[16][16], r3[16][16];
        // (0) forward: k_step2 order vs the three-MFMA composition
        {
            std::vector<Blk> s2;
            for (int c = 0; c < NCH; ++c) {
                s2.push_back(hh[c]);
                s2.push_back(hl[c]);
                s2.push_back(lh[c]);
            }
            R.go32(s2, bias, r2);
            std::vector<std::pair<const Blk*, const Blk*>> s3;
            for (int s = 0; s < NCH / 2; ++s) {
                s3.push_back({&hh[2 * s], &hl[2 * s]});
                s3.push_back({&lh[2 * s], &hh[2 * s + 1]});
                s3.push_back({&hl[2 * s + 1], &lh[2 * s + 1]});
            }
            R.go16(s3, bias, r3);
            tot[0] += ndiff(r2, r3);
            outs[0] += 256;
        }
        // (1) forward with an odd chunk count (5 chunks: layer 0 at L = 16): the last pair's second half zero
        {
            std::vector<Blk> s2;
            for (int c = 0; c < 5; ++c) {
                s2.push_back(hh[c]);
                s2.push_back(hl[c]);
                s2.push_back(lh[c]);
            }
            R.go32(s2, bias, r2);
            std::vector<std::pair<const Blk*, const Blk*>> s3;
            for (int s = 0; s < 3; ++s) {
                const bool two = 2 * s + 1 < 5;
                s3.push_back({&hh[2 * s], &hl[2 * s]});
                s3.push_back({&lh[2 * s], two ? &hh[2 * s + 1] : nullptr});
                if (two) s3.push_back({&hl[2 * s + 1], &lh[2 * s + 1]});
            }
            R.go16(s3, bias, r3);
            tot[1] += ndiff(r2, r3);
            outs[1] += 256;
        }
        // (2) dgrad: [hd(c) | ld(c)] vs hd(c), ld(c); from zero
        {
            float z[16][16] = {};
            std::vector<Blk> s2;
            for (int c = 0; c < NCH; ++c) {
                s2.push_back(hd[c]);
                s2.push_back(ld[c]);
            }
            R.go32(s2, z, r2);
            std::vector<std::pair<const Blk*, const Blk*>> s3;
            for (int c = 0; c < NCH; ++c) s3.push_back({&hd[c], &ld[c]});
            R.go16(s3, z, r3);
            tot[2] += ndiff(r2, r3);
            outs[2] += 256;
        }
        // (4) dgrad from ONE register D = [dz(2s) | dz(2s+1)] with the B lane-group pattern:
        //     [hd(2s) | ld(2s)] with blgp 1 (lanes 0-31 into 32-63), [hd(2s+1) | ld(2s+1)] with blgp 2
        {
            float z[16][16] = {};
            std::vector<Blk> s2;
            for (int c = 0; c < NCH; ++c) {
                s2.push_back(hd[c]);
                s2.push_back(ld[c]);
            }
            R.go32(s2, z, r2);
            std::vector<std::pair<const Blk*, const Blk*>> s3, b3;
            std::vector<int> g;
            for (int s = 0; s < NCH / 2; ++s) {
                s3.push_back({&hd[2 * s], &ld[2 * s]});
                b3.push_back({&hd[2 * s], &hd[2 * s + 1]});  // the B fragment as the register holds it
                g.push_back(1);
                s3.push_back({&hd[2 * s + 1], &ld[2 * s + 1]});
                b3.push_back({&hd[2 * s], &hd[2 * s + 1]});
                g.push_back(2);
            }
            R.go16(s3, z, r3, &b3, &g);
            tot[4] += ndiff(r2, r3);
            outs[4] += 256;
        }
        // (3) dW_last: one K = 32 16x16x32 MFMA from zero vs two chained halves
        {
            float z[16][16] = {};
            const Blk& t0 = hd[0];
            const Blk& t1 = hd[1];
            std::vector<std::pair<const Blk*, const Blk*>> one = {{&t0, &t1}};
            R.go16(one, z, r2);
            float x[16][16];
            std::vector<std::pair<const Blk*, const Blk*>> first = {{&t0, nullptr}}, second = {{nullptr, &t1}};
            R.go16(first, z, x);
            R.go16(second, x, r3);
            tot[3] += ndiff(r2, r3);
            outs[3] += 256;
        }
    }
    const char* names[5] = {"forward 3-term composition (16 chunks)", "forward, 5 chunks (odd tail)",
                            "dgrad [hd|ld] composition", "K=32 split into two chained halves",
                            "dgrad from one register, blgp 1 / 2"};
    for (int i = 0; i < 5; ++i) printf("%-42s: %lld of %lld outputs differ\n", names[i], tot[i], outs[i]);
    return 0;
}
