// microbench.hip -- FP64 instruction throughput on MI355X (the guides list no FP64 rates).
// Each kernel runs a dependent-free stream of one operation over 8 independent chains per
// lane; reports ns per wave-instruction and the implied cycles at the measured clock.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;
constexpr int CH = 8;

template <int OP>
__global__ __launch_bounds__(256) void kbench(double* out, double seed) {
  double v[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) v[c] = seed + 0.001 * (threadIdx.x + c);
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (OP == 0) v[c] = fma(v[c], 0.999999, 1e-7);                      // v_fma_f64
      if (OP == 1) v[c] = __builtin_amdgcn_rcp(v[c]);                       // v_rcp_f64
      if (OP == 2) v[c] = 1.0 / v[c];                                       // IEEE division sequence
      if (OP == 3) v[c] = exp(v[c] * 1e-3) ;                                // ocml exp (+mul)
      if (OP == 4) v[c] = sqrt(v[c]);                                       // IEEE sqrt sequence
      if (OP == 5) { double r = __builtin_amdgcn_rcp(v[c]);                 // rcp + 2 Newton
                     double e = fma(-v[c], r, 1.0); r = fma(r, e, r);
                     e = fma(-v[c], r, 1.0); v[c] = fma(r, e, r); }
      if (OP == 6) v[c] = __builtin_amdgcn_rsq(v[c]);                       // v_rsq_f64
      if (OP == 7) v[c] = (float)(1.0f / (float)v[c]);                      // f32 rcp + cvts
      if (OP == 8) v[c] = ldexp(v[c], (int)(threadIdx.x & 1) - (int)(c & 1)); // v_ldexp_f64
      if (OP == 9) v[c] = v[c] * 0.999999;                                  // v_mul_f64
      if (OP == 10) v[c] = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, v[c]) ^ 1ull); // 2x v_xor_b32
      if (OP == 11) { v[c] = (double)__builtin_amdgcn_rsqf((float)v[c]); asm volatile("" : "+v"(v[c])); }  // cvt + v_rsq_f32 + cvt
      if (OP == 12) v[c] = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, v[c]) & 0xFFFFFFFFFFFFF7FFull); // 1x v_and_b32
      if (OP == 13) { v[c] = (double)(float)v[c]; asm volatile("" : "+v"(v[c])); }  // cvt f64->f32 + cvt f32->f64
      if (OP == 14) v[c] = __builtin_sqrt(v[c]);                                 // sqrt (IEEE) again as reference
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// float-only chains: v_rsq_f32 (OP 0), v_fma_f32 (OP 1)
template <int OP>
__global__ __launch_bounds__(256) void kbenchf(double* out, float seed) {
  float v[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) v[c] = seed + 0.001f * (threadIdx.x + c);
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      if (OP == 0) v[c] = __builtin_amdgcn_rsqf(v[c]);
      if (OP == 1) v[c] = fmaf(v[c], 0.999999f, 1e-7f);
    }
  }
  float s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// accuracy of raw v_rcp_f64 and rcp+NR vs correctly rounded division
__global__ void kacc(const double* x, double* e_raw, double* e_nr, double* e_rsq, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double d = x[i], q = 1.0 / d, r = __builtin_amdgcn_rcp(d);
  e_raw[i] = fabs(r - q) / q;
  double e = fma(-d, r, 1.0); double r1 = fma(r, e, r); e = fma(-d, r1, 1.0); r1 = fma(r1, e, r1);
  e_nr[i] = fabs(r1 - q) / q;
  double s = 1.0 / sqrt(d), rs = __builtin_amdgcn_rsq(d);
  e_rsq[i] = fabs(rs - s) / s;
  // f32 rsq estimate, one FP64 Newton step (the modified lanes' sqrt form: g = X y, v = 1.5 - 0.5 g y, sqrt = g v)
  double y32 = (double)__builtin_amdgcn_rsqf((float)d);
  double g = d * y32, v = fma(-0.5, g * y32, 1.5), sq = sqrt(d);
  e_raw[i + n] = fabs(g * v - sq) / sq;
  double y64 = rs, g6 = d * y64, v6 = fma(-0.5, g6 * y64, 1.5);
  e_raw[i + 2 * n] = fabs(g6 * v6 - sq) / sq;
}

template <int OP, bool F = false>
float run(double* out, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  if (F) hipLaunchKernelGGL(kbenchf<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.5f);
  else hipLaunchKernelGGL(kbench<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.5);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) {
    if (F) hipLaunchKernelGGL(kbenchf<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.5f);
    else hipLaunchKernelGGL(kbench<OP>, dim3(blocks), dim3(256), 0, 0, out, 1.5);
  }
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  int blocks = 256 * 8;   // 8 blocks of 4 waves per CU
  double* out;
  hipMalloc(&out, sizeof(double) * blocks * 256);
  const char* names[] = {"v_fma_f64", "v_rcp_f64", "1.0/x (IEEE)", "exp(x) ocml", "sqrt (IEEE)", "rcp+2NR", "v_rsq_f64",
                         "f32 rcp+cvt", "v_ldexp_f64", "v_mul_f64", "2x v_xor_b32", "cvt+rsq_f32+cvt",
                         "v_and_b32", "2x cvt", "sqrt (IEEE)", "v_rsq_f32", "v_fma_f32"};
  const int NOPS = 17;
  float ms[NOPS];
  ms[0] = run<0>(out, blocks); ms[1] = run<1>(out, blocks); ms[2] = run<2>(out, blocks); ms[3] = run<3>(out, blocks);
  ms[4] = run<4>(out, blocks); ms[5] = run<5>(out, blocks); ms[6] = run<6>(out, blocks); ms[7] = run<7>(out, blocks);
  ms[8] = run<8>(out, blocks); ms[9] = run<9>(out, blocks); ms[10] = run<10>(out, blocks);
  ms[11] = run<11>(out, blocks); ms[12] = run<12>(out, blocks); ms[13] = run<13>(out, blocks);
  ms[14] = run<14>(out, blocks); ms[15] = run<0, true>(out, blocks); ms[16] = run<1, true>(out, blocks);
  const double ops = (double)blocks * 4 /*waves*/ * ITERS * CH;   // wave-level operations
  const double simds = 256 * 4;
  for (int k = 0; k < NOPS; k++) {
    const double ns_per_op_per_simd = ms[k] * 1e6 / (ops / simds);
    printf("%-14s %8.3f ms  %6.3f ns/wave-op/SIMD  (= %.1f cycles @2.4GHz, %.2fx fma)\n", names[k], ms[k],
           ns_per_op_per_simd, ns_per_op_per_simd * 2.4, ms[k] / ms[0]);
  }
  const int n = 1 << 20;
  double *x, *e1, *e2, *e3;
  hipMalloc(&x, n * 8); hipMalloc(&e1, 3 * n * 8); hipMalloc(&e2, n * 8); hipMalloc(&e3, n * 8);
  double* hx = new double[n];
  unsigned long long s = 88172645463325252ull;
  for (int i = 0; i < n; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; hx[i] = 1e-3 + (double)(s % 1000000007ull) * 1e-4; }
  hipMemcpy(x, hx, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(kacc, dim3(n / 256), dim3(256), 0, 0, x, e1, e2, e3, n);
  double* h1 = new double[3 * n]; double* h2 = new double[n]; double* h3 = new double[n];
  hipMemcpy(h1, e1, 3 * n * 8, hipMemcpyDeviceToHost); hipMemcpy(h2, e2, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h3, e3, n * 8, hipMemcpyDeviceToHost);
  double m1 = 0, m2 = 0, m3 = 0;
  for (int i = 0; i < n; i++) { if (h1[i] > m1) m1 = h1[i]; if (h2[i] > m2) m2 = h2[i]; if (h3[i] > m3) m3 = h3[i]; }
  printf("max rel err: raw v_rcp_f64 %.3e   rcp+2NR %.3e   raw v_rsq_f64 %.3e\n", m1, m2, m3);
  double m4 = 0, m5 = 0;
  for (int i = 0; i < n; i++) { if (h1[n + i] > m4) m4 = h1[n + i]; if (h1[2 * n + i] > m5) m5 = h1[2 * n + i]; }
  printf("max rel err of sqrt as g v after one FP64 Newton step: from v_rsq_f32 %.3e   from v_rsq_f64 %.3e\n", m4, m5);
  return 0;
}
