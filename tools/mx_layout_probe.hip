// Operand-layout probe for the block-scaled MX MFMA on gfx950
// (__builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4, A/B = OCP fp8 e4m3, e8m0 block scales).
// Hypothesis (by analogy with mfma_f32_32x32x16_bf16): lane l holds A[row l & 31][k = 32 (l >> 5) + j]
// and B[k = 32 (l >> 5) + j][col l & 31] in byte j = 0..31 of its 8 VGPRs, and the lane's scale byte
// applies to those 32 k values. The probe fills A, B with small integers (exact in e4m3) and
// per-lane scales 2^s, runs one MFMA and compares with a host product; prints PASS/FAIL counts.
// Build: hipcc --offload-arch=gfx950 -O2 tools/mx_layout_probe.hip -o mx_layout_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

// OCP e4m3fn encoding of a small integer-valued float (|v| <= 448, exact values only)
static unsigned char e4m3(float v) {
  if (v == 0.f) return 0;
  unsigned char s = v < 0 ? 0x80 : 0;
  float a = std::fabs(v);
  int e = (int)std::floor(std::log2(a));
  float mant = a / std::ldexp(1.f, e) - 1.f;  // [0, 1)
  int m = (int)std::lround(mant * 8.f);
  if (m == 8) { m = 0; ++e; }
  return (unsigned char)(s | ((e + 7) << 3) | m);
}

__global__ void probe(const unsigned char* A, const unsigned char* B, const unsigned char* sa, const unsigned char* sb,
                      float* D) {
  const int l = threadIdx.x;
  v8i a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    pa[j] = A[(l & 31) * 64 + 32 * (l >> 5) + j];   // A row-major [32][64]
    pb[j] = B[(32 * (l >> 5) + j) * 32 + (l & 31)];  // B row-major [64][32]
  }
  v16f c = {};
  const int sca = sa[l], scb = sb[l];
  // cbsz = 0 / blgp = 0: fp8 e4m3 operands; opsel 0: scale byte 0 of the VGPR
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sca, 0, scb);
  for (int r = 0; r < 16; ++r) {
    const int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
    D[row * 32 + col] = c[r];
  }
}

int main() {
  std::vector<float> Af(32 * 64), Bf(64 * 32);
  std::vector<unsigned char> A(32 * 64), B(64 * 32), sa(64), sb(64);
  srand(7);
  for (int i = 0; i < 32 * 64; ++i) {
    Af[i] = (float)(rand() % 9 - 4);
    A[i] = e4m3(Af[i]);
  }
  for (int i = 0; i < 64 * 32; ++i) {
    Bf[i] = (float)((rand() % 7) - 3) * (i % 3 == 0 ? 2.f : 1.f);
    B[i] = e4m3(Bf[i]);
  }
  // per-lane scales: lane l of A covers row l & 31, k half l >> 5; exponents 0 / +1 / -1
  int ea[64], eb[64];
  for (int l = 0; l < 64; ++l) {
    ea[l] = (l * 5) % 3 - 1;
    eb[l] = (l * 7) % 3 - 1;
    sa[l] = (unsigned char)(127 + ea[l]);
    sb[l] = (unsigned char)(127 + eb[l]);
  }
  std::vector<double> ref(32 * 32, 0.0);
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double acc = 0.0;
      for (int k = 0; k < 64; ++k) {
        const int la = i + 32 * (k / 32), lb = j + 32 * (k / 32);
        acc += Af[i * 64 + k] * std::ldexp(1.0, ea[la]) * Bf[k * 32 + j] * std::ldexp(1.0, eb[lb]);
      }
      ref[i * 32 + j] = acc;
    }
  unsigned char *dA, *dB, *dsa, *dsb;
  float* dD;
  hipMalloc(&dA, A.size());
  hipMalloc(&dB, B.size());
  hipMalloc(&dsa, 64);
  hipMalloc(&dsb, 64);
  hipMalloc(&dD, 32 * 32 * sizeof(float));
  hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  hipMemcpy(dsa, sa.data(), 64, hipMemcpyHostToDevice);
  hipMemcpy(dsb, sb.data(), 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsa, dsb, dD);
  std::vector<float> D(32 * 32);
  hipMemcpy(D.data(), dD, D.size() * sizeof(float), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32 * 32; ++i)
    if (std::fabs(D[i] - ref[i]) > 1e-3 * (1.0 + std::fabs(ref[i]))) {
      if (bad < 5) printf("mismatch at (%d,%d): got %g want %g\n", i / 32, i % 32, D[i], ref[i]);
      ++bad;
    }
  printf("%s: %d of 1024 mismatches\n", bad ? "FAIL" : "PASS", bad);
  return bad ? 1 : 0;
}
