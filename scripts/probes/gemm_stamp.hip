// Probe: per-workgroup timeline of one pg_gemm_f32 launch (start/end wall clock at 100 MHz,
// shader clocks, XCC / CU / SIMD of each workgroup). Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -DPG_GEMM_STAMP=1 -Iinclude \
//     -Ipla-gnn_amd/csrc scripts/probes/gemm_stamp.hip -o scripts/probes/gemm_stamp_probe
// Usage: gemm_stamp_probe ta tb M N K [x]   (prints a summary; stamps to stamps.csv)
#include "gemm.hip"

#include <algorithm>
#include <cstdarg>
#include <string>
#include <vector>

namespace pg {
char* error_buffer() { static char b[256]; return b; }
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fprintf(stderr, "\n");
  return code;
}
}  // namespace pg

int main(int argc, char** argv) {
  if (argc < 6) return 2;
  const int ta = atoi(argv[1]), tb = atoi(argv[2]);
  const int64_t M = atoll(argv[3]), N = atoll(argv[4]), K = atoll(argv[5]);
  const char* csv = argc > 6 ? argv[6] : "stamps.csv";
  float *A, *B, *C;
  (void)hipMalloc(&A, M * K * 4);
  (void)hipMalloc(&B, N * K * 4);
  (void)hipMalloc(&C, M * N * 4);
  std::vector<float> h(std::max(M, N) * K);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  (void)hipMemcpy(A, h.data(), M * K * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(B, h.data(), N * K * 4, hipMemcpyHostToDevice);
  const int64_t lda = ta ? M : K, ldb = tb ? K : N;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int warm = getenv("WARM") ? atoi(getenv("WARM")) : 5;
  for (int i = 0; i < warm; ++i) pg_gemm_f32(ta, tb, M, N, K, 1.f, A, lda, B, ldb, 0.f, C, N, nullptr, 1, nullptr, 0, nullptr);
  (void)hipEventRecord(e0);
  const int rc = pg_gemm_f32(ta, tb, M, N, K, 1.f, A, lda, B, ldb, 0.f, C, N, nullptr, 1, nullptr, 0, nullptr);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st(65536 * 4);
  (void)hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(pg_gemm_stamp), st.size() * 8);
  int bm, bn;
  pick_tile(M, N, K, 1, bm, bn);
  const int tiles = (int)(((M + bm - 1) / bm) * ((N + bn - 1) / bn));
  unsigned long long t0 = ~0ull, t1 = 0;
  double ck = 0, dur = 0;
  for (int b = 0; b < tiles && b < 65536; ++b) {
    t0 = std::min(t0, st[4 * b]);
    t1 = std::max(t1, st[4 * b + 1]);
    dur += (st[4 * b + 1] - st[4 * b]) * 10.0;  // ns
    ck += st[4 * b + 2];
  }
  printf("rc %d  %ldx%ldx%ld ta %d tb %d tile %dx%d blocks %d  event %.1f us  span %.1f us  "
         "mean block %.1f us  clock %.2f GHz  %.1f TF\n",
         rc, (long)M, (long)N, (long)K, ta, tb, bm, bn, tiles, ms * 1e3, (t1 - t0) / 100.0,
         dur / tiles / 1e3, ck / (dur), 2.0 * M * N * K / (ms * 1e-3) / 1e12);
  std::vector<unsigned long long> ks(64 * 64);
  (void)hipMemcpyFromSymbol(ks.data(), HIP_SYMBOL(pg_gemm_kstamp), ks.size() * 8);
  {
    std::string kp = std::string(csv) + ".ksteps";
    FILE* g = fopen(kp.c_str(), "w");
    const int nk = (int)std::min<int64_t>(64, (K + 31) / 32);
    for (int b = 0; b < 64 && b < tiles; ++b) {
      for (int t = 1; t < nk; ++t) fprintf(g, "%llu ", ks[b * 64 + t] - ks[b * 64 + t - 1]);
      fprintf(g, "\n");
    }
    fclose(g);
  }
  {
    std::vector<unsigned long long> ph(64 * 4);
    (void)hipMemcpyFromSymbol(ph.data(), HIP_SYMBOL(pg_gemm_kphase), ph.size() * 8);
    std::vector<double> pro, loop, epi;
    for (int b = 0; b < 64 && b < tiles; ++b) {
      pro.push_back((double)(ph[b * 4 + 1] - ph[b * 4]));
      loop.push_back((double)(ph[b * 4 + 2] - ph[b * 4 + 1]));
      epi.push_back((double)(ph[b * 4 + 3] - ph[b * 4 + 2]));
    }
    auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    printf("   phases (median clocks, first 64 blocks): prologue %.0f  loop %.0f  epilogue %.0f\n",
           med(pro), med(loop), med(epi));
  }
  FILE* f = fopen(csv, "w");
  fprintf(f, "block,start_ns,end_ns,clocks,xcc,hw_id\n");
  for (int b = 0; b < tiles && b < 65536; ++b)
    fprintf(f, "%d,%llu,%llu,%llu,%llu,%llu\n", b, (st[4 * b] - t0) * 10, (st[4 * b + 1] - t0) * 10,
            st[4 * b + 2], st[4 * b + 3] >> 32, st[4 * b + 3] & 0xffffffffull);
  fclose(f);
  return 0;
}
