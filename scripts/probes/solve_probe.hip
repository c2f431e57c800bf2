// Probe of batch_solve (als_batch.hip) alone: NM SPD systems of size KP per wave, built on the
// host, loaded straight into the accumulator layout; prints the max relative error of x vs a
// host Cholesky solve for each (KP, NM).  Standalone binary (includes the kernel source).
#include "../../csrc/kernels/als_batch.hip"
#include <cmath>
#include <cstdio>
#include <vector>

template <int KP, int NM>
__global__ void probe(const float* A, const float* b, float* x, float* dbg) {
  constexpr int M = KP / 16, NT = M * (M + 1) / 2;
  __shared__ __attribute__((aligned(16))) float smem[NM * 16 * BATCH_DS + NM * 16 + 64];
  const int lane = threadIdx.x & 63, g = lane >> 4, f = lane & 15;
  f32x4 acc[NM][NT];
  float bpart[NM][M], cnt[NM];
  int slot[NM];
  bool valid[NM];
  for (int m = 0; m < NM; ++m) {
    const float* Am = A + (size_t)m * KP * KP;
    for (int pi = 0; pi < M; ++pi)
      for (int qi = pi; qi < M; ++qi)
        for (int v = 0; v < 4; ++v)
          acc[m][tix<M>(pi, qi)][v] = Am[(16 * pi + 4 * g + v) * KP + 16 * qi + f];
    for (int pi = 0; pi < M; ++pi) bpart[m][pi] = g == 0 ? b[m * KP + 16 * pi + f] : 0.f;
    cnt[m] = 0.f;
    slot[m] = -1;
    valid[m] = true;
  }
  oryx_als::AlsParams p{};
  p.k = KP;
  p.lambda = 0.f;
  lds_float* scr = (lds_float*)smem;
  lds_float* vdis = scr + NM * 16 * BATCH_DS;
  float xs[M];
  batch_solve<KP, NM>(p, lane, acc, bpart, cnt, slot, valid, scr, vdis, xs, [](auto) {},
                      [](int) {});
  for (int pp = 0; pp < M; ++pp) x[(size_t)lane * M + pp] = xs[pp];
  (void)dbg;
}

template <int KP, int NM>
void run() {
  const int n = KP;
  std::vector<float> A(NM * n * n), b(NM * n);
  unsigned s = 12345 + KP * 7 + NM;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0 - 0.5; };
  for (int m = 0; m < NM; ++m) {
    std::vector<double> X(3 * n * n);
    for (auto& v : X) v = rnd();
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        double acc = i == j ? 1.0 : 0.0;
        for (int t = 0; t < 3 * n; ++t) acc += X[t * n + i] * X[t * n + j];
        A[m * n * n + i * n + j] = (float)acc;
      }
    for (int i = 0; i < n; ++i) b[m * n + i] = (float)rnd();
  }
  float *dA, *db, *dx, *dd;
  (void)hipMalloc(&dA, A.size() * 4);
  (void)hipMalloc(&db, b.size() * 4);
  (void)hipMalloc(&dx, 64 * (KP / 16) * 4);
  (void)hipMalloc(&dd, 4096 * 4);
  (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemset(dx, 0xff, 64 * (KP / 16) * 4);
  hipLaunchKernelGGL((probe<KP, NM>), dim3(1), dim3(64), 0, 0, dA, db, dx, dd);
  const hipError_t le = hipGetLastError();
  const hipError_t se = hipDeviceSynchronize();
  std::vector<float> xs(64 * (KP / 16));
  (void)hipMemcpy(xs.data(), dx, xs.size() * 4, hipMemcpyDeviceToHost);
  if (le != hipSuccess || se != hipSuccess)
    printf("KP=%d NM=%d launch %s sync %s\n", KP, NM, hipGetErrorString(le), hipGetErrorString(se));
  double worst = 0;
  for (int m = 0; m < NM; ++m) {
    // host Cholesky solve in double
    std::vector<double> L(n * n, 0.0), y(n), xr(n);
    for (int j = 0; j < n; ++j) {
      double d = A[m * n * n + j * n + j];
      for (int k = 0; k < j; ++k) d -= L[j * n + k] * L[j * n + k];
      L[j * n + j] = std::sqrt(d);
      for (int i = j + 1; i < n; ++i) {
        double v = A[m * n * n + i * n + j];
        for (int k = 0; k < j; ++k) v -= L[i * n + k] * L[j * n + k];
        L[i * n + j] = v / L[j * n + j];
      }
    }
    for (int i = 0; i < n; ++i) {
      double v = b[m * n + i];
      for (int k = 0; k < i; ++k) v -= L[i * n + k] * y[k];
      y[i] = v / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
      double v = y[i];
      for (int k = i + 1; k < n; ++k) v -= L[k * n + i] * xr[k];
      xr[i] = v / L[i * n + i];
    }
    double num = 0, den = 0;
    for (int g = 0; g < 4; ++g) {
      if (g % NM != m) continue;
      for (int i = 0; i < n; ++i) {
        const int lane = g * 16 + (i & 15), pp = i / 16;
        const double d = xs[lane * (KP / 16) + pp] - xr[i];
        num += d * d;
        den += xr[i] * xr[i];
      }
    }
    const double rel = std::sqrt(num / den);
    if (m == 0) printf("  x[0..2] = %g %g %g  ref %g %g %g\n", xs[0], xs[(KP / 16)], xs[2 * (KP / 16)], xr[0], xr[1], xr[2]);
    if (rel > worst) worst = rel;
  }
  printf("KP=%3d NM=%d max rel err %.3e\n", KP, NM, worst);
}

int main() {
  run<16, 4>(); run<16, 2>(); run<16, 1>();
  run<32, 2>(); run<64, 4>(); run<64, 2>(); run<64, 1>();
  run<128, 1>();
  return 0;
}
