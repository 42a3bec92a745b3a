// Host side of the prefill GEMM (gemm_pf.h): which launches it serves and the tile / split-K plan.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "gemm_pf.h"

namespace aios {

extern template bool pf_launch_fmt<QT_Q4_K, QT_Q4_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q6_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q4_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_BF16, QT_BF16>(const GemmQArgs&, int, int, int, hipStream_t);

static int pf_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

struct PfPlan {
  int bm = 0, bn = 0, s = 1;
};

// Modelled time of one launch.  Per workgroup: max(MFMA time at the tile's sustained fraction of the
// per-CU peak, its slot bytes at the per-CU L2 gather rate) + a fixed prologue / epilogue; a grid
// larger than the chip runs in rounds (one workgroup per CU: the slots fill the LDS); split-K adds
// its fp32 atomic traffic (and the zeroing of a STORE target).
static double pf_model(const GemmQArgs& a, int bm, int bn, int S, bool bf) {
  const double cus = device_cu_count();
  const double tiles = (double)((a.M + bm - 1) / bm) * (a.N / bn);
  const double ksteps = (double)(a.K / 64) / S;
  // sustained MFMA fraction per tile shape (dequant VALU + LDS fragment reads beside the MFMAs)
  double eff = bm == 256 ? 0.55 : (bm == 128 ? 0.48 : 0.32);
  if (bn == 128) eff *= 0.85;
  const double t_mfma = 2.0 * bm * bn * 64 * ksteps / (eff * 9.6e12);
  const double slot = bm * 128.0 + bn * (bf ? 128.0 : 48.0);
  const double t_mem = slot * ksteps / 55e9;
  const double t_wg = std::max(t_mfma, t_mem) + 2.5e-6;
  double t = std::ceil(tiles * S / cus) * t_wg;
  if (S > 1) t += (double)a.M * a.N * 4 * S / 1.2e12 + (a.epi == GEPI_STORE ? (double)a.M * a.N * 4 / 4e12 : 0.0);
  return t;
}

static bool pf_tile_ok(const GemmQArgs& a, int bn) {
  if (a.N % bn) return false;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % bn || a.seg[s].rows % bn) return false;
  return true;
}

static PfPlan pf_plan(const GemmQArgs& a, bool bf) {
  PfPlan best;
  double bt = 1e30;
  // AIOS_GEMM_PF_TILE=BMxBN / AIOS_GEMM_PF_SPLIT=S pin the plan (sweeps: tools/bench_gemm.py --pf-sweep)
  // (read per call: tests and sweeps change them inside one process)
  const char* tile = std::getenv("AIOS_GEMM_PF_TILE");
  const int split = pf_env("AIOS_GEMM_PF_SPLIT", 0);
  int fbm = 0, fbn = 0;
  if (tile) std::sscanf(tile, "%dx%d", &fbm, &fbn);
  const int nk = a.K / 64;
  for (int bm : {256, 128, 64}) {
    for (int bn : {256, 128}) {
      if (fbm && (bm != fbm || bn != fbn)) continue;
      if (!pf_tile_ok(a, bn)) continue;
      for (int S : {1, 2, 3, 4, 6, 8, 12, 16}) {
        if (a.ksplit > 0 && S != a.ksplit) continue;
        if (a.ksplit <= 0 && split > 0 && S != split) continue;
        if (S > 1 && (a.epi == GEPI_SWIGLU_BF16 || nk / S < 2)) continue;
        const double t = pf_model(a, bm, bn, S, bf);
        if (t < bt) {
          bt = t;
          best.bm = bm; best.bn = bn; best.s = S;
        }
      }
    }
  }
  return best;
}

// Serves M >= AIOS_GEMM_PF_MIN_M (default 33: the ring GEMM keeps 5..32) for Q4_K / Q6_K / mixed
// Q4_K|Q6_K / bf16 weight stacks with the STORE / ACCUM / SWIGLU epilogues; false -> the caller's
// fallback (formats and fused epilogues this kernel does not do).
bool launch_gemm_pf(const GemmQArgs& a, hipStream_t st) {
  const int on = pf_env("AIOS_GEMM_PF", 1);
  const int min_m = pf_env("AIOS_GEMM_PF_MIN_M", 33);
  if (!on || a.M < min_m || a.nseg < 1) return false;
  if (a.epi != GEPI_STORE && a.epi != GEPI_ACCUM && a.epi != GEPI_SWIGLU_BF16) return false;
  if (a.nrm_in || a.lda % 8 || ((uintptr_t)a.A & 15)) return false;
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  for (int s = 0; s + 1 < a.nseg; ++s)
    if (a.seg[s].qtype != qt0) return false;
  const bool bf = qt0 == QT_BF16;
  if (bf ? (qt1 != QT_BF16 || a.K % 64) : (a.K % 256)) return false;
  if (!bf && !((qt0 == QT_Q4_K || qt0 == QT_Q6_K) && (qt1 == QT_Q4_K || qt1 == QT_Q6_K))) return false;
  if (qt0 == QT_Q6_K && qt1 == QT_Q4_K) return false;  // not instantiated (no such stack in the GGUF recipes)
  if (a.epi == GEPI_SWIGLU_BF16 && (!a.C16 || a.nseg != 1)) return false;
  if (a.epi != GEPI_SWIGLU_BF16 && !a.C) return false;
  const PfPlan p = pf_plan(a, bf);
  if (!p.bm) return false;
  if (p.s > 1 && a.epi == GEPI_STORE)
    HIP_CHECK(hipMemset2DAsync(a.C, (size_t)a.ldc * 4, 0, (size_t)a.N * 4, a.M, st));
  if (qt0 == QT_Q4_K && qt1 == QT_Q4_K) return pf_launch_fmt<QT_Q4_K, QT_Q4_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q6_K && qt1 == QT_Q6_K) return pf_launch_fmt<QT_Q6_K, QT_Q6_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q4_K && qt1 == QT_Q6_K) return pf_launch_fmt<QT_Q4_K, QT_Q6_K>(a, p.bm, p.bn, p.s, st);
  return pf_launch_fmt<QT_BF16, QT_BF16>(a, p.bm, p.bn, p.s, st);
}

// the plan the launcher would pick (bindings / tools)
void gemm_pf_plan(const GemmQArgs& a, int& bm, int& bn, int& s) {
  const PfPlan p = pf_plan(a, a.seg[0].qtype == QT_BF16);
  bm = p.bm; bn = p.bn; s = p.s;
}

}  // namespace aios
