// Host side of the prefill GEMM (gemm_pf.h): which launches it serves and the tile / split-K plan.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <mutex>
#include <tuple>
#include <vector>

#include "gemm_pf.h"

namespace aios {

extern template bool pf_launch_fmt<QT_Q4_K, QT_Q4_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q6_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q4_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_BF16, QT_BF16>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q5_K, QT_Q5_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q5_K, QT_Q6_K>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q4_0, QT_Q4_0>(const GemmQArgs&, int, int, int, hipStream_t);
extern template bool pf_launch_fmt<QT_Q8_0, QT_Q8_0>(const GemmQArgs&, int, int, int, hipStream_t);

static int pf_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

struct PfPlan {
  int bm = 0, bn = 0, s = 1;  // s < 0: stream-K over the CUs (gemm_pf.h pf_stream_k)
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
  if (S < 0) {  // stream-K: every CU the same share of the tile x K-step iterations, ~2 partial tiles each
    const double iters = tiles * (a.K / 64.0), per = std::ceil(iters / cus);
    const double t_it = std::max(t_mfma, t_mem) / ksteps;
    return per * t_it + 2 * 2.5e-6 + (double)cus * 2 * bm * bn * 4 / 1.2e12 +
           (a.epi == GEPI_STORE ? (double)a.M * a.N * 4 / 4e12 : 0.0);
  }
  double t = std::ceil(tiles * S / cus) * t_wg;
  const double R = std::fmod(tiles, cus);
  if (bm == 256 && S == 1 && (bn == 128 || !bf) && tiles > cus && R > 0 && 2 * R <= cus)  // tail split
    t = (std::floor(tiles / cus) + 0.6) * t_wg;
  if (S > 1) t += (double)a.M * a.N * 4 * S / 1.2e12 + (a.epi == GEPI_STORE ? (double)a.M * a.N * 4 / 4e12 : 0.0);
  return t;
}

static bool pf_tile_ok(const GemmQArgs& a, int bn) {
  if (a.N % bn) return false;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % bn || a.seg[s].rows % bn) return false;
  return true;
}

// Measured plans: one per (shape, formats, epilogue, M bucket), filled by gemm_pf_autotune (the
// engine tunes its projection shapes at finalize); the model below is the fallback.
using PfKey = std::tuple<int, int, int, int, int, int, int, int, int, int>;
static int pf_bucket(int M) {
  int b = 64;
  while (b < M && b < 2048) b <<= 1;
  return M > 2048 ? (M + 2047) / 2048 * 2048 : b;
}
static PfKey pf_key(const GemmQArgs& a) {
  // (+ the CU budget: a CU-masked co-resident engine plans for its own CUs)
  return PfKey(a.N, a.K, pf_bucket(a.M), a.epi, a.seg[0].qtype, a.seg[a.nseg - 1].qtype, a.nseg,
               a.nseg > 1 ? a.seg_n0[1] : 0, a.nseg > 2 ? a.seg_n0[2] : 0, device_cu_count());
}
static std::mutex pf_mu;
static std::map<PfKey, PfPlan>& pf_tuned() {
  static std::map<PfKey, PfPlan> m;
  return m;
}
// the best plan without split-K per key (GEPI_QKV launches: the RoPE / KV-cache epilogue cannot
// take split partials; they use the STORE shape's tuned S = 1 plan -- tuning them for real would
// write the KV cache)
static std::map<PfKey, PfPlan>& pf_tuned_s1() {
  static std::map<PfKey, PfPlan> m;
  return m;
}
// AIOS_GEMM_PF_DETERMINISTIC=1: no split-K / stream-K plans (their fp32 atomics add partial tiles in
// arrival order, so the low bits of a prefill could differ run to run even with the same plan)
static bool pf_deterministic() { return pf_env("AIOS_GEMM_PF_DETERMINISTIC", 0) != 0; }
static bool pf_no_split(const GemmQArgs& a) {
  return a.epi == GEPI_SWIGLU_BF16 || a.epi == GEPI_QKV || pf_deterministic();
}
// stream-K: STORE / ACCUM launches whose tiles leave CUs idle, with an even K-step count per tile
// (every stream-K segment then spans >= 2 steps / 256-blocks); AIOS_GEMM_PF_SK=0 keeps it out of plans
static bool pf_sk_ok(const GemmQArgs& a, int bm, int bn, bool bf) {
  if (pf_no_split(a) || !pf_env("AIOS_GEMM_PF_SK", 1)) return false;
  const int units = bn == 256 && !bf ? a.K / 256 : a.K / 64;
  const double tiles = (double)((a.M + bm - 1) / bm) * (a.N / bn);
  return units % 2 == 0 && units >= 4 && tiles < 2.0 * device_cu_count();
}

// every plan the launcher could run for these args (ksplit > 0 pins the split)
static std::vector<PfPlan> pf_candidates(const GemmQArgs& a, bool bf) {
  std::vector<PfPlan> out;
  const int nk = a.K / 64;
  for (int bm : {256, 128, 64})
    for (int bn : {256, 128}) {
      if (!pf_tile_ok(a, bn)) continue;
      for (int S : {1, 2, 3, 4, 6, 8, 12, 16, -1}) {
        if (a.ksplit > 0 && S != a.ksplit) continue;
        if (S < 0 && !pf_sk_ok(a, bm, bn, bf)) continue;
        if (S > 1 && (pf_no_split(a) || nk / S < 2)) continue;
        if (!bf && bn == 256 && (a.K / 256) / S < 1) continue;
        PfPlan p;
        p.bm = bm; p.bn = bn; p.s = S;
        out.push_back(p);
      }
    }
  return out;
}

static PfPlan pf_model_plan(const GemmQArgs& a, bool bf, bool s1_only);
static PfPlan pf_plan(const GemmQArgs& a, bool bf) {
  if (!std::getenv("AIOS_GEMM_PF_TILE") && !std::getenv("AIOS_GEMM_PF_SPLIT") && a.ksplit <= 0) {
    std::lock_guard<std::mutex> g(pf_mu);
    if (a.epi == GEPI_QKV || pf_deterministic()) {  // (the best plan without split partials)
      GemmQArgs b = a;
      if (a.epi == GEPI_QKV) b.epi = GEPI_STORE;
      auto it = pf_tuned_s1().find(pf_key(b));
      if (it != pf_tuned_s1().end()) return it->second;
    } else {
      auto it = pf_tuned().find(pf_key(a));
      if (it != pf_tuned().end()) return it->second;
    }
  }
  return pf_model_plan(a, bf, false);
}

// the modelled plan (pf_model), or the one AIOS_GEMM_PF_TILE / _SPLIT / a.ksplit pin
static PfPlan pf_model_plan(const GemmQArgs& a, bool bf, bool s1_only) {
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
      for (int S : {1, 2, 3, 4, 6, 8, 12, 16, -1}) {
        if (a.ksplit > 0 && S != a.ksplit) continue;
        if (a.ksplit <= 0 && split != 0 && S != split) continue;  // (AIOS_GEMM_PF_SPLIT=-1: stream-K)
        if (S < 0 && (s1_only || !pf_sk_ok(a, bm, bn, bf))) continue;
        if (S > 1 && (s1_only || pf_no_split(a) || nk / S < 2)) continue;
        if (!bf && bn == 256 && (a.K / 256) / S < 1) continue;  // pf8c slices whole 256-blocks
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

// Serves M >= AIOS_GEMM_PF_MIN_M (default 33: the ring GEMM keeps 5..32) for Q4_K / Q5_K / Q6_K / mixed
// Q4_K|Q6_K, Q5_K|Q6_K / Q4_0 / Q8_0 / bf16 weight stacks with the STORE / ACCUM / SWIGLU epilogues; false -> the caller's
// fallback (formats and fused epilogues this kernel does not do).
static bool pf_eligible(const GemmQArgs& a);
static bool pf_run(const GemmQArgs& a, const PfPlan& p, hipStream_t st) {
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  if (p.s != 1 && a.epi == GEPI_QKV) return false;  // (plans keep S = 1 for it; a pinned split declines)
  if (p.s != 1 && a.epi == GEPI_STORE)
    HIP_CHECK(hipMemset2DAsync(a.C, (size_t)a.ldc * 4, 0, (size_t)a.N * 4, a.M, st));
  if (qt0 == QT_Q4_K && qt1 == QT_Q4_K) return pf_launch_fmt<QT_Q4_K, QT_Q4_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q6_K && qt1 == QT_Q6_K) return pf_launch_fmt<QT_Q6_K, QT_Q6_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q4_K && qt1 == QT_Q6_K) return pf_launch_fmt<QT_Q4_K, QT_Q6_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q5_K && qt1 == QT_Q5_K) return pf_launch_fmt<QT_Q5_K, QT_Q5_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q5_K && qt1 == QT_Q6_K) return pf_launch_fmt<QT_Q5_K, QT_Q6_K>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q4_0 && qt1 == QT_Q4_0) return pf_launch_fmt<QT_Q4_0, QT_Q4_0>(a, p.bm, p.bn, p.s, st);
  if (qt0 == QT_Q8_0 && qt1 == QT_Q8_0) return pf_launch_fmt<QT_Q8_0, QT_Q8_0>(a, p.bm, p.bn, p.s, st);
  if (qt0 != QT_BF16) return false;
  return pf_launch_fmt<QT_BF16, QT_BF16>(a, p.bm, p.bn, p.s, st);
}

bool launch_gemm_pf(const GemmQArgs& a, hipStream_t st) {
  const int on = pf_env("AIOS_GEMM_PF", 1);
  const int min_m = pf_env("AIOS_GEMM_PF_MIN_M", 33);
  if (!on || a.M < min_m) return false;
  if (!pf_eligible(a)) return false;
  const PfPlan p = pf_plan(a, a.seg[0].qtype == QT_BF16);
  if (!p.bm) return false;
  return pf_run(a, p, st);
}

static bool pf_eligible(const GemmQArgs& a) {
  if (a.nseg < 1 || a.M < 1) return false;
  if (a.epi != GEPI_STORE && a.epi != GEPI_ACCUM && a.epi != GEPI_SWIGLU_BF16 && a.epi != GEPI_QKV) return false;
  if (a.epi == GEPI_QKV && (a.kv_fp8 || a.col0 != 0 || !a.q_out || !a.k_cache || !a.v_cache || !a.pos || !a.rope_cs ||
                            a.head_dim % 2 || a.N != a.q_dim + 2 * a.kv_dim))
    return false;
  if (a.nrm_in || a.lda % 8 || ((uintptr_t)a.A & 15)) return false;
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  for (int s = 0; s + 1 < a.nseg; ++s)
    if (a.seg[s].qtype != qt0) return false;
  const bool bf = qt0 == QT_BF16;
  if (bf ? (qt1 != QT_BF16 || a.K % 64) : (a.K % 256)) return false;
  // instantiated stacks (gemm_pf_*.hip): the GGUF recipes' Q4_K_M / Q5_K_M (mixed QKV: Q|K Q4_K or Q5_K, V Q6_K),
  // Q6_K, Q4_0 and Q8_0 matrices
  const bool kq = (qt0 == QT_Q4_K && (qt1 == QT_Q4_K || qt1 == QT_Q6_K)) || (qt0 == QT_Q6_K && qt1 == QT_Q6_K) ||
                  (qt0 == QT_Q5_K && (qt1 == QT_Q5_K || qt1 == QT_Q6_K)) || (qt0 == QT_Q4_0 && qt1 == QT_Q4_0) ||
                  (qt0 == QT_Q8_0 && qt1 == QT_Q8_0);
  if (!bf && !kq) return false;
  if (a.epi == GEPI_SWIGLU_BF16 && (!a.C16 || a.nseg != 1)) return false;
  if (a.epi != GEPI_SWIGLU_BF16 && a.epi != GEPI_QKV && !a.C) return false;
  return true;
}

// Time every candidate plan for these args (real buffers; outputs overwritten) and keep the fastest
// for their M bucket.  Returns the number of candidates timed (0: not a prefill-GEMM launch, or a
// key already planned in this process -- tuned by an earlier engine or imported, gemm_pf_import: a
// second engine never changes the plans a first one runs).
//
// Stable choice: a measured plan replaces the modelled one only when it is > 5 % faster,
// so timing noise (a co-tenant, TP ranks sharing the GPU) does not pick a different tile / split in
// each process; ties keep the earlier candidate (a fixed order).  TP ranks then take rank 0's plans
// (tp.py broadcasts gemm_pf_export), and AIOS_GEMM_PF_PLANS persists them across processes.
int gemm_pf_autotune(const GemmQArgs& a, hipStream_t st) {
  if (!pf_eligible(a)) return 0;
  {
    std::lock_guard<std::mutex> g(pf_mu);
    if (pf_tuned().count(pf_key(a))) return 0;
  }
  const bool bf = a.seg[0].qtype == QT_BF16;
  const std::vector<PfPlan> cands = pf_candidates(a, bf);
  if (cands.empty()) return 0;
  const PfPlan mp = pf_model_plan(a, bf, false), mp1 = pf_model_plan(a, bf, true);
  float tm = -1.f, tm1 = -1.f;  // the modelled plans' measured times
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  PfPlan best = cands[0], best1 = cands[0];
  float bt = 1e30f, bt1 = 1e30f;
  for (const PfPlan& p : cands) {
    pf_run(a, p, st);  // warm (code object load, caches)
    HIP_CHECK(hipEventRecord(e0, st));
    for (int r = 0; r < 3; ++r) pf_run(a, p, st);
    HIP_CHECK(hipEventRecord(e1, st));
    HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < bt) {
      bt = ms;
      best = p;
    }
    if (p.s == 1 && ms < bt1) {  // (stream-K is not an S = 1 plan either)
      bt1 = ms;
      best1 = p;
    }
    auto same = [](const PfPlan& x, const PfPlan& y) { return x.bm == y.bm && x.bn == y.bn && x.s == y.s; };
    if (same(p, mp)) tm = ms;
    if (same(p, mp1)) tm1 = ms;
  }
  HIP_CHECK(hipEventDestroy(e0));
  HIP_CHECK(hipEventDestroy(e1));
  if (tm > 0.f && bt > 0.95f * tm) best = mp;
  if (tm1 > 0.f && bt1 > 0.95f * tm1) best1 = mp1;
  std::lock_guard<std::mutex> g(pf_mu);
  pf_tuned()[pf_key(a)] = best;
  if (bt1 < 1e30f) pf_tuned_s1()[pf_key(a)] = best1;
  return (int)cands.size();
}

// every tuned plan as flat ints: 10 key fields, bm, bn, s, map (0: best, 1: best without split-K)
std::vector<int> gemm_pf_export() {
  std::lock_guard<std::mutex> g(pf_mu);
  std::vector<int> v;
  for (int m = 0; m < 2; ++m)
    for (const auto& kv : (m ? pf_tuned_s1() : pf_tuned())) {
      const PfKey& k = kv.first;
      for (int x : {std::get<0>(k), std::get<1>(k), std::get<2>(k), std::get<3>(k), std::get<4>(k), std::get<5>(k),
                    std::get<6>(k), std::get<7>(k), std::get<8>(k), std::get<9>(k)})
        v.push_back(x);
      v.push_back(kv.second.bm); v.push_back(kv.second.bn); v.push_back(kv.second.s); v.push_back(m);
    }
  return v;
}

// install plans (replacing any tuned for the same keys): TP workers take the leader's, a process
// takes a persisted set; later autotune calls skip these keys
void gemm_pf_import(const std::vector<int>& v) {
  if (v.size() % 14) throw std::runtime_error("gemm_pf_import: bad plan list");
  std::lock_guard<std::mutex> g(pf_mu);
  for (size_t i = 0; i < v.size(); i += 14) {
    const PfKey k(v[i], v[i + 1], v[i + 2], v[i + 3], v[i + 4], v[i + 5], v[i + 6], v[i + 7], v[i + 8], v[i + 9]);
    PfPlan p;
    p.bm = v[i + 10]; p.bn = v[i + 11]; p.s = v[i + 12];
    (v[i + 13] ? pf_tuned_s1() : pf_tuned())[k] = p;
  }
}

// whether launch_gemm_pf takes these args (the engine asks before choosing the GEPI_QKV epilogue
// for a prefill chunk, which only this kernel and the small-M ones implement)
bool gemm_pf_serves(const GemmQArgs& a) {
  if (!pf_env("AIOS_GEMM_PF", 1) || a.M < pf_env("AIOS_GEMM_PF_MIN_M", 33) || !pf_eligible(a)) return false;
  const PfPlan p = pf_plan(a, a.seg[0].qtype == QT_BF16);
  return p.bm != 0 && !(p.s != 1 && a.epi == GEPI_QKV);
}

// the plan the launcher would pick (bindings / tools)
void gemm_pf_plan(const GemmQArgs& a, int& bm, int& bn, int& s) {
  const PfPlan p = pf_plan(a, a.seg[0].qtype == QT_BF16);
  bm = p.bm; bn = p.bn; s = p.s;
}

}  // namespace aios
