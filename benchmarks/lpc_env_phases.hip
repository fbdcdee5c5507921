// Microbenchmark: time of the LPC stage kernels (launch_lpc_env: Durbin + cepstrum + envelope) alone on the
// WSJ shape (327680 items = 4096 frames x 80 bands, p = 150, M = 100, 150 envelope samples) or REVERB's M:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I speech_recognition_tools_amd/csrc \
//         benchmarks/lpc_env_phases.hip -o benchmarks/lpc_env_p7
// r is the autocorrelation of an AR(2) process.  (The round-3/4 per-phase splits of DESIGN.md §6 came from
// phase masks compiled into the kernel then; the product kernel no longer carries them.)
#include "../speech_recognition_tools_amd/csrc/fdlp_lpc.hip"

#include <math.h>
#include <stdio.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
  const int items = argc > 1 ? atoi(argv[1]) : 327680;
  const int M = argc > 2 ? atoi(argv[2]) : 100;  // coeff_num: 100 (WSJ / CHiME-4), 450 (REVERB)
  const int p = 150, nlags = 152, kk = 150, env_nfft = 300;
  std::vector<double> r((size_t)items * nlags);
  for (int it = 0; it < items; ++it) {
    // AR(2) autocorrelation with a per-item pole: r_l = rho^l cos(w l), plus a white floor
    const double rho = 0.90 + 0.08 * ((it * 37) % 101) / 100.0, w = 0.2 + 2.5 * ((it * 13) % 97) / 97.0;
    for (int l = 0; l < nlags; ++l) r[(size_t)it * nlags + l] = pow(rho, l) * cos(w * l) + (l == 0 ? 1e-3 : 0.0);
  }
  std::vector<double> weights(3 * M, 1.0), cosv(env_nfft), win(2 * kk);
  for (int q = 0; q < env_nfft; ++q) cosv[q] = cos(2 * M_PI * q / env_nfft);
  for (int t = 0; t < kk; ++t) {
    win[2 * t] = 0.5 - 0.5 * cos(2 * M_PI * t / (kk - 1));
    win[2 * t + 1] = 0.54 - 0.46 * cos(2 * M_PI * t / (kk - 1));
  }
  win[0] = 0.0; win[1] = 0.08;
  double *d_r, *d_w, *d_cos, *d_win, *d_env;
  CK(hipMalloc(&d_r, r.size() * 8));
  CK(hipMalloc(&d_w, weights.size() * 8));
  CK(hipMalloc(&d_cos, cosv.size() * 8));
  CK(hipMalloc(&d_win, win.size() * 8));
  CK(hipMalloc(&d_env, (size_t)items * kk * 8));
  CK(hipMemcpy(d_r, r.data(), r.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_w, weights.data(), weights.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_cos, cosv.data(), cosv.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_win, win.data(), win.size() * 8, hipMemcpyHostToDevice));
  fdlp::DevConsts c{};
  c.p = p; c.nlags = nlags; c.M = M; c.Me = M < env_nfft ? M : env_nfft; c.kk = kk; c.env_nfft = env_nfft;
  c.weights = d_w; c.env_cos = d_cos; c.env_win = d_win;
  CK(fdlp::prepare_lpc_env(c));  // lattice kernel launch geometry (FDLP_LPC_SLOTMAJOR / FDLP_LPC_LDS read here)
  double *d_a, *d_gg;  // split Durbin workspace (durbin8_kernel)
  CK(hipMalloc(&d_a, (size_t)items * (c.lpc_astride > p + 1 ? c.lpc_astride : p + 1) * 8));
  CK(hipMalloc(&d_gg, (size_t)items * 8));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (int i = 0; i < 3; ++i) CK(fdlp::launch_lpc_env(c, 0, d_r, items, d_env, nullptr, nullptr, nullptr, d_a, d_gg, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(fdlp::launch_lpc_env(c, 0, d_r, items, d_env, nullptr, nullptr, nullptr, d_a, d_gg, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<double> env((size_t)kk * 4);
  CK(hipMemcpy(env.data(), d_env, env.size() * 8, hipMemcpyDeviceToHost));
  double cs = 0;
  for (double v : env) cs += v;
  printf("lpc_env items=%d M=%d: %.4f ms/launch (checksum %.6e)\n", items, M, ms / reps, cs);
  return 0;
}
