// C ABI of the MoEvA2 engine (see include/moeva_mi355x.h for the contract and the
// reference surfaces each entry point replaces).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <numeric>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/moeva_mi355x.h"
#include "check.h"
#include "detmath.h"
#include "engine.h"
#include "kernels.h"
#include "rowops.h"

using namespace mv;

namespace mv {
thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;  // kernels.h MV_LAUNCH
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                    \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(MV_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
  } while (0)

template <class T>
hipError_t dalloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc((void**)p, n * sizeof(T));
  // MV_POISON=<byte>: fill every new device buffer (development check for reads of memory
  // nothing wrote: results must not change)
  static const char* poison = std::getenv("MV_POISON");
  if (e == hipSuccess && poison)
    e = hipMemset(*p, std::atoi(poison) & 0xFF, n * sizeof(T));
  return e;
}

template <class T>
hipError_t upload(T** p, const T* host, size_t n) {
  hipError_t e = dalloc(p, n);
  if (e != hipSuccess) return e;
  if (n && host) return hipMemcpy(*p, host, n * sizeof(T), hipMemcpyHostToDevice);
  return hipSuccess;
}

__global__ void k_fill_d(double* p, size_t n, double v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ void k_fill_i(int* p, size_t n, int v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// True unless `p` is known device memory of a GPU other than `dev` (host or unregistered
// pointers pass: the kernels' own faults report those).  Entry points taking buffers of
// another GPU would otherwise run on `dev` with peer pointers and no cross-device order.
bool on_device(const void* p, int dev) {
  if (!p) return true;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return true;
  }
  return at.type != hipMemoryTypeDevice || at.device == dev;
}

}  // namespace

// fp32 -> bf16 bits, round to nearest even (NaN stays a quiet NaN)
static unsigned short bf16_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (unsigned short)((u >> 16) | 0x40);
  return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

// Host copy of the problem and model descriptors: the engine builds its device tables from
// it at creation (every gene stored) and again at mv_set_states for the compact layout.
struct HostProblem {
  int D = 0, V = 0, Dm = 0, C = 0, n_ohe = 0, n_pool = 0, norm = 2, scale_obj = 1;
  double tol = 0.0;
  std::vector<int> kind, feat, ohe_off, ohe_feats, mut, op_code, op_arg, pool;
  std::vector<double> op_k, mls, mlm;
};
struct HostModel {
  int n_layers = 0;
  int dims[MAX_LAYERS + 1] = {};
  std::vector<float> W[MAX_LAYERS], b[MAX_LAYERS];
};

struct mv_engine {
  int device = 0;
  int mlp_bf16 = 0;  // bf16 perf mode of the classifier tiles (mv_set_mlp_precision)
  HostProblem hp;
  HostModel hm;
  DProblem p{};      // every gene stored: mv_evaluate / mv_decode / mv_variation, hosted loops
  std::vector<void*> prob_allocs;
  // The attack's layout for the current state set (mv_set_states): compact when some genes
  // can never change in any of the states (integer genes with xl == xu == their initial
  // value); those are not stored in the pool, moved, mutated or summed.  ap() / as() / ag0()
  // are what mv_attack_run reads.
  bool compact = false;
  std::vector<int> stored;           // the compact layout's stored genes
  // mv_set_gene_layout: the layout the next mv_set_states uses (empty: derive it from the
  // bound batch); a caller that splits one job into batches passes the whole job's layout
  std::vector<int> layout_req;
  DProblem pc{};
  std::vector<void*> compact_allocs;  // pc's tables (kept while the stored set is unchanged)
  DStates sc{};
  double* genes0c = nullptr;
  std::vector<void*> cstate_allocs;
  const DProblem& ap() const { return compact ? pc : p; }
  const DStates& as() const { return compact ? sc : s; }
  double* ag0() const { return compact ? genes0c : genes0; }
  float* W1full = nullptr;
  float* b1 = nullptr;
  int H1 = 0;
  // states
  int B = 0;
  std::vector<void*> state_allocs;
  DStates s{};
  double* genes0 = nullptr;
  // attack
  std::vector<void*> attack_allocs;
  int P = 0, O = 0, S = 0, n_gen = 0, R = 0, hist_mode = 0, hist_w = 0, hist_rows = 0;
  double* pool = nullptr;
  double* poolF = nullptr;
  int* pop_slot = nullptr;
  int* free_slot = nullptr;
  int* parents = nullptr;
  // k_genc attacks: the variation plan k_survive writes for the next generation (VPlan)
  bool has_plan = false;
  int4* plan_hdr = nullptr;
  int* plan_mw = nullptr;
  double* plan_mu = nullptr;
  double *ideal = nullptr, *worst = nullptr, *extreme = nullptr;
  int* has_ext = nullptr;
  double* ref = nullptr;
  std::vector<double> ref_host;  // the reference points currently in e->ref
  double* hist = nullptr;
  // mv_attack_front scratch when the caller passes no mask / offsets (attack_allocs)
  unsigned char* front_scr = nullptr;
  int* off_scr = nullptr;
  bool attack_ready = false;
  bool has_model = false;
  long long* d_phase = nullptr;  // MV_SURV_PHASES=1: survival phase clocks [B][16]
  long long* d_gphase = nullptr; // MV_GEN_PHASES=1: k_genc clocks [grid][8] (one group)
  bool gphase_mlp = false;        // MV_MLP_PHASES=1: the same buffer holds the classifier's
  size_t gphase_n = 0;
  unsigned long long* dom_g = nullptr;  // P + O > SURV_NLDS: survival dominance bitsets
  size_t dom_stride = 0;
  float* xml = nullptr;  // k_vary -> k_mlp scratch
  size_t xml_cap = 0;
  hipError_t ensure_xml(size_t rows) {
    const size_t need = rows * (size_t)p.Dm4;
    if (need <= xml_cap) return hipSuccess;
    if (xml) (void)hipFree(xml);
    xml = nullptr;
    xml_cap = 0;
    hipError_t e = dalloc(&xml, need);
    if (e == hipSuccess) xml_cap = need;
    return e;
  }
  // state-group streams (index 0 = the caller's stream, not owned)
  hipStream_t streams[MAX_GROUPS] = {};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_join[MAX_GROUPS] = {};
  hipError_t ensure_streams(int n) {
    hipError_t err = hipSuccess;
    if (!ev_fork) err = hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming);
    for (int q = 1; q < n && err == hipSuccess; ++q) {
      if (!streams[q]) err = hipStreamCreateWithFlags(&streams[q], hipStreamNonBlocking);
      if (err == hipSuccess && !ev_join[q])
        err = hipEventCreateWithFlags(&ev_join[q], hipEventDisableTiming);
    }
    return err;
  }
  // profiling
  int cx_kind = 0;          // 0: two-point (reference), 1: SBX
  double sbx_eta = 30.0, cx_prob = 0.9;
  int state_keys = 0;       // mv_set_state_streams: state b draws from stream key0 + b
  uint32_t key0 = 0;
  int attack_mode = 0;      // 0: auto, 1: per-phase chain (the only schedule)
  bool profiling = false;
  std::vector<hipEvent_t> ev_var, ev_cons, ev_mlp, ev_surv;
  // kernel-exact profiling pairs per recorded generation: k_gen(c) start / stop, k_cons start /
  // stop, classifier start / stop (hipExtLaunchKernelGGL stamps, kernels.h MV_LAUNCH); the
  // survival pair is ev_surv
  std::vector<hipEvent_t> ev_kx;
  int n_var_rec = 0, n_surv_rec = 0;

  void free_list(std::vector<void*>& v) {
    for (void* x : v) (void)hipFree(x);
    v.clear();
  }
  template <class T>
  hipError_t keep(std::vector<void*>& list, T** p, const T* host, size_t n) {
    hipError_t e = upload(p, host, n);
    if (e == hipSuccess) list.push_back((void*)*p);
    return e;
  }
  ~mv_engine() {
    (void)hipSetDevice(device);
    if (xml) (void)hipFree(xml);
    free_list(attack_allocs);
    free_list(cstate_allocs);
    free_list(state_allocs);
    free_list(compact_allocs);
    free_list(prob_allocs);
    for (auto e : ev_var) (void)hipEventDestroy(e);
    for (auto e : ev_mlp) (void)hipEventDestroy(e);
    for (auto e : ev_cons) (void)hipEventDestroy(e);
    for (int q = 1; q < MAX_GROUPS; ++q) {
      if (streams[q]) (void)hipStreamDestroy(streams[q]);
      if (ev_join[q]) (void)hipEventDestroy(ev_join[q]);
    }
    if (ev_fork) (void)hipEventDestroy(ev_fork);
    for (auto e : ev_surv) (void)hipEventDestroy(e);
    for (auto e : ev_kx) (void)hipEventDestroy(e);
    (void)hipGetLastError();  // do not leave a teardown status for the next launch check
  }
};

// The device tables of one gene layout.  keep: the stored genes (ascending indices into the
// problem's V genes), or empty for all of them.  The draws stay defined over all V genes
// (Vr, the gap table, the crossover subsets' sizes and every gene's subset index); cmap /
// fidx (region B) translate.  A kept subset is only built for IDENT problems, where the
// dropped genes' features are then simply immutable features: decoded from x_init, folded
// into the per-state layer-1 bias, absent from f2's sum.
static int build_problem(const HostProblem& h, const HostModel* hm, const std::vector<int>& keep,
                         DProblem& p, std::vector<void*>& allocs) {
  const int Vr = h.V, D = h.D, C = h.C;
  std::vector<int> gk(keep);
  if (gk.empty()) {
    gk.resize(Vr);
    std::iota(gk.begin(), gk.end(), 0);
  }
  const int V = (int)gk.size();
  std::vector<int> sub_full(Vr), cmap(Vr, -1);
  int ns[2] = {0, 0};
  for (int g = 0; g < Vr; ++g) sub_full[g] = ns[h.kind[g] == MV_GENE_REAL ? 0 : 1]++;
  std::vector<int> kind(V), feat(V), sub(V);
  for (int c = 0; c < V; ++c) {
    kind[c] = h.kind[gk[c]];
    feat[c] = h.feat[gk[c]];
    sub[c] = sub_full[gk[c]];
    cmap[gk[c]] = c;
  }
  std::vector<int> mut(h.mut);
  if ((int)gk.size() < Vr) mut = feat;  // IDENT: stored gene c <-> mutable feature c
  const int Dm = (int)mut.size();
  p = DProblem{};
  p.D = D;
  p.V = V;
  p.Vr = Vr;
  p.compact = V < Vr;
  p.Dm = Dm;
  p.Dm4 = (Dm + 15) & ~15;  // mutable features padded to a 16-k MFMA group
  p.C = C;
  p.n_ohe = h.n_ohe;
  p.n_sub[0] = ns[0];
  p.n_sub[1] = ns[1];
  const int n_ohe_feats = h.n_ohe > 0 ? h.ohe_off[h.n_ohe] : 0;
  p.n_ohe_feat = n_ohe_feats;
  hipError_t err = hipSuccess;
  auto K = [&](auto** dst, const auto* host, size_t n) {
    if (err != hipSuccess) return;
    err = upload(dst, host, n);
    if (err == hipSuccess) allocs.push_back((void*)*dst);
  };
  K((int**)&p.gene_kind, kind.data(), V);
  K((int**)&p.gene_feat, feat.data(), V);
  K((int**)&p.gene_sub, sub.data(), V);
  const int V4 = (V + 3) & ~3;
  std::vector<int> info(V4, 0);
  for (int c = 0; c < V; ++c) info[c] = kind[c] | (sub[c] << 2) | (feat[c] << 17);
  K((int**)&p.gene_info, info.data(), V4);
  K((int**)&p.ohe_off, h.ohe_off.data(), h.ohe_off.size());
  K((int**)&p.ohe_feat, h.ohe_feats.data(), n_ohe_feats);
  K((int**)&p.mut_feat, mut.data(), Dm);
  {  // feature -> gene map of the decoder (mv_decode): -1 immutable, gene | (category+1) << 16
    std::vector<int> fdec(D, -1);
    for (int c = 0; c < V; ++c) {
      if (kind[c] != MV_GENE_OHE) {
        if (feat[c] >= 0 && feat[c] < D) fdec[feat[c]] = c;
      } else {
        const int q = feat[c];
        for (int k = h.ohe_off[q]; k < h.ohe_off[q + 1]; ++k)
          if (h.ohe_feats[k] >= 0 && h.ohe_feats[k] < D)
            fdec[h.ohe_feats[k]] = c | ((k - h.ohe_off[q] + 1) << 16);
      }
    }
    K((int**)&p.fdec, fdec.data(), D);
  }
  K((double**)&p.ml_scale, h.mls.data(), D);
  K((double**)&p.ml_min, h.mlm.data(), D);
  std::vector<double> ms(p.Dm4, 0.0), mm(p.Dm4, 0.0);
  for (int j = 0; j < Dm; ++j) {
    ms[j] = h.mls[mut[j]];
    mm[j] = h.mlm[mut[j]];
  }
  K((double**)&p.mlS, ms.data(), p.Dm4);
  K((double**)&p.mlM, mm.data(), p.Dm4);
  // constraint program sorted by op code (lane-uniform branches), ABS_SUMDIFF ops last
  std::vector<int> order(C);
  for (int c = 0; c < C; ++c) order[c] = c;
  auto key = [&](int c) { return h.op_code[c] == MV_OP_ABS_SUMDIFF ? 1 << 20 : h.op_code[c]; };
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key(x) < key(y); });
  std::vector<int> scode(C), sarg((size_t)C * 4), scol(C);
  std::vector<double> sk((size_t)C * 2);
  int n_sd = 0;
  for (int k = 0; k < C; ++k) {
    const int c = order[k];
    scode[k] = h.op_code[c];
    scol[k] = c;
    for (int q = 0; q < 4; ++q) sarg[(size_t)k * 4 + q] = h.op_arg[(size_t)c * 4 + q];
    for (int q = 0; q < 2; ++q) sk[(size_t)k * 2 + q] = h.op_k[(size_t)c * 2 + q];
    n_sd += scode[k] == MV_OP_ABS_SUMDIFF;
  }
  K((int**)&p.op_code, scode.data(), C);
  K((int**)&p.op_arg, sarg.data(), (size_t)C * 4);
  K((double**)&p.op_k, sk.data(), (size_t)C * 2);
  K((int**)&p.op_col, scol.data(), C);
  K((int**)&p.idx_pool, h.pool.data(), h.n_pool);
  p.n_pool = h.n_pool;
  p.n_sumdiff = n_sd;
  p.full_ops = 0;
  for (int c = 0; c < C; ++c)
    if (h.op_code[c] >= MV_OP_LCLD_INSTALL && h.op_code[c] <= MV_OP_RATIO_MASKED) p.full_ops = 1;
  p.ident = V == Dm;
  for (int c = 0; c < V && p.ident; ++c) p.ident = kind[c] != MV_GENE_OHE && feat[c] == mut[c];
  {  // k_vary problem blob: the LDS image of the tables (kernels.h vary_offsets)
    const VaryOff vo = vary_offsets(p);
    if (gen_lds(vo, false, false, true).total > 160 * 1024 || cons_lds_total(vo) > 160 * 1024)
      return fail(MV_ERR_ARG, "problem too large for the k_vary LDS workspace");
    std::vector<unsigned char> blob(vo.vb, 0);
    auto put = [&](unsigned off, const void* src, size_t n) {
      if (n) std::memcpy(blob.data() + off, src, n);
    };
    put(vo.opa, sarg.data(), (size_t)C * 16);
    put(vo.opk, sk.data(), (size_t)C * 16);
    put(vo.mlS, ms.data(), (size_t)p.Dm4 * 8);
    put(vo.mlM, mm.data(), (size_t)p.Dm4 * 8);
    put(vo.opc, scode.data(), (size_t)C * 4);
    put(vo.ocol, scol.data(), (size_t)C * 4);
    put(vo.pool, h.pool.data(), (size_t)h.n_pool * 4);
    put(vo.ginfo, info.data(), (size_t)V4 * 4);
    put(vo.mutf, mut.data(), (size_t)Dm * 4);
    put(vo.ooff, h.ohe_off.data(), h.ohe_off.size() * 4);
    if (n_ohe_feats > 0) put(vo.ofeat, h.ohe_feats.data(), (size_t)n_ohe_feats * 4);
    put(vo.cmap, cmap.data(), (size_t)Vr * 4);
    put(vo.fidx, gk.data(), (size_t)V * 4);
    // mutation gap table T[k] = floor((1 - 1/Vr)^k 2^32), k = 0..Vr (oracle geometric_table)
    std::vector<uint32_t> geo(Vr + 1);
    const double q = 1.0 - 1.0 / (double)Vr;
    for (int k = 0; k <= Vr; ++k) {
      const double t = std::floor(std::pow(q, (double)k) * 4294967296.0);
      geo[k] = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
    }
    put(vo.geo, geo.data(), (size_t)(Vr + 1) * 4);
    {  // region S: k_genc's slim program (kernels.h); the packed words mirror rowops pack_op
      // with SlotRow operands: slot j < Dm = stored mutable feature j (the wave's row buffer),
      // Dm + f = feature f of x_init (IDENT problems: k_genc's only ones)
      const int n_lane = C - n_sd;
      // tol >= 0: constraints_slim's clamp (v <= tol ? 0 : v) equals the general one then
      p.slim = p.ident && n_lane <= 64 * OPS_REG && Dm + D < 0x4000 && h.tol >= 0.0;
      std::vector<int> slot(D);
      for (int f = 0; f < D; ++f) slot[f] = Dm + f;
      for (int j = 0; j < Dm; ++j) slot[mut[j]] = j;
      auto sl = [&](int f) { return f >= 0 && f < D ? slot[f] : 0; };
      std::vector<double> k1(C);
      std::vector<int> sd((size_t)(n_sd > 0 ? n_sd : 1) * 4, 0);
      std::vector<unsigned> opw(C);
      bool sd_small = true;  // every ABS_SUMDIFF side within one term per lane
      for (int k = 0; k < C; ++k) {
        k1[k] = sk[(size_t)k * 2];
        const int* ar = &sarg[(size_t)k * 4];
        if (k < n_lane) {
          p.slim &= (scode[k] == MV_OP_DIFF || scode[k] == MV_OP_RATIO_SAFE) && ar[0] >= 0 &&
                    ar[0] < D && ar[1] >= 0 && ar[1] < D;
          opw[k] = (unsigned)scode[k] | ((unsigned)sl(ar[0]) << 4) | ((unsigned)sl(ar[1]) << 18);
        } else {
          opw[k] = 0u;
          for (int q = 0; q < 4; ++q) sd[(size_t)(k - n_lane) * 4 + q] = ar[q];
          sd_small &= ar[1] - ar[0] <= 64 && ar[2] - ar[1] <= 64;
        }
      }
      p.sd_reg = p.slim && n_sd <= SD_REG && sd_small;
      std::vector<int> spool(h.n_pool > 0 ? h.n_pool : 1, 0);
      for (int q = 0; q < h.n_pool; ++q) {
        p.slim &= h.pool[q] >= 0 && h.pool[q] < D;
        spool[q] = sl(h.pool[q]);
      }
      put(vo.s_k, k1.data(), (size_t)C * 8);
      put(vo.s_col, scol.data(), (size_t)C * 4);
      put(vo.s_pool, spool.data(), (size_t)h.n_pool * 4);
      put(vo.s_sd, sd.data(), sd.size() * 4);
      put(vo.s_opw, opw.data(), (size_t)C * 4);
      if (std::getenv("MV_SLIM") && std::getenv("MV_SLIM")[0] == '0') p.slim = 0;  // A/B
      if (!p.slim || (std::getenv("MV_SD_REG") && std::getenv("MV_SD_REG")[0] == '0'))
        p.sd_reg = 0;
    }
    K((unsigned char**)&p.vblob, blob.data(), blob.size());
  }
  p.tol = h.tol;
  p.norm = h.norm;
  p.scale_obj = h.scale_obj;
  p.f2_scale = h.norm == 2 ? 1.0 / (std::sqrt((double)D) - 0.0) : 1.0;
  if (hm) {
    p.n_layers = hm->n_layers;
    for (int l = 0; l <= hm->n_layers; ++l) p.dims[l] = hm->dims[l];
    const int H1 = hm->dims[1];
    // layer 0: mutable rows, zero padded to Dm4
    std::vector<float> w1m((size_t)p.Dm4 * H1, 0.f);
    for (int j = 0; j < Dm; ++j)
      std::memcpy(&w1m[(size_t)j * H1], hm->W[0].data() + (size_t)mut[j] * H1, H1 * sizeof(float));
    K((float**)&p.W[0], w1m.data(), w1m.size());
    for (int l = 1; l < hm->n_layers; ++l) {
      K((float**)&p.W[l], hm->W[l].data(), (size_t)hm->dims[l] * hm->dims[l + 1]);
      K((float**)&p.bias[l], hm->b[l].data(), hm->dims[l + 1]);
    }
    // k_mlp2 packing of the hidden layers: Wp[kg][n][16] = W[16 kg + i][n] (zero padded)
    p.mlp2 = 1;
    for (int l = 1; l < hm->n_layers; ++l) p.mlp2 &= hm->dims[l] % 16 == 0 && hm->dims[l] <= 128;
    // xml_direct: k_mlp2 builds its layer-0 tiles from the child genes (MV_XML: the fp32
    // ML rows written by the row kernel + k_mlp2, A/B only)
    p.xml_direct = p.mlp2 && p.ident && !std::getenv("MV_XML");
    // the same packing feeds k_mlpw32 (fp32 wide nets): every hidden width a multiple of 16
    bool pack16 = true;
    for (int l = 1; l < hm->n_layers; ++l) pack16 &= hm->dims[l] % 16 == 0;
    for (int l = 0; l + 1 < hm->n_layers && pack16; ++l) {
      const int Kl = l == 0 ? p.Dm4 : hm->dims[l], Nl = hm->dims[l + 1];
      const float* src = l == 0 ? w1m.data() : hm->W[l].data();  // [Kl][Nl] row-major
      std::vector<float> wp((size_t)Kl * Nl, 0.f);
      for (int k = 0; k < Kl; ++k)
        for (int n = 0; n < Nl; ++n)
          wp[((size_t)(k / 16) * Nl + n) * 16 + (k % 16)] = src[(size_t)k * Nl + n];
      K((float**)&p.Wp[l], wp.data(), wp.size());
    }
    // bf16 perf mode packing of the MFMA layers: Wb[kg][n][32] = bf16(W[32 kg + i][n]), K
    // zero padded to a multiple of 32 (engine.h DProblem::Wb)
    for (int l = 0; l + 1 < hm->n_layers; ++l) {
      const int Kl = l == 0 ? p.Dm4 : hm->dims[l], Nl = hm->dims[l + 1];
      const int K32 = (Kl + 31) & ~31;
      const float* src = l == 0 ? w1m.data() : hm->W[l].data();  // [Kl][Nl] row-major
      std::vector<unsigned short> wb((size_t)K32 * Nl, 0);
      for (int k = 0; k < Kl; ++k)
        for (int n = 0; n < Nl; ++n)
          wb[((size_t)(k / 32) * Nl + n) * 32 + (k % 32)] = bf16_bits(src[(size_t)k * Nl + n]);
      K((unsigned short**)&p.Wb[l], wb.data(), wb.size());
    }
  } else {
    p.n_layers = 0;
  }
  if (err != hipSuccess) return fail(MV_ERR_HIP, std::string("upload: ") + hipGetErrorString(err));
  if (hm) {
    int hmax = 16;
    for (int l = 1; l < p.n_layers; ++l) hmax = p.dims[l] > hmax ? p.dims[l] : hmax;
    // the attack's classifier tiles (k_mlp / k_mlp2) read the mutable features only
    const size_t lds = mlp_lds_bytes(p.Dm4, hmax, p.dims[p.n_layers - 1], p.dims[p.n_layers]);
    if (lds > 160 * 1024) return fail(MV_ERR_ARG, "problem too large for the evaluation tile (LDS)");
  }
  return MV_OK;
}

extern "C" {

const char* mv_last_error(void) { return g_err.c_str(); }

int mv_device_count(int32_t* n) {
  int c = 0;
  HIPCHK(hipGetDeviceCount(&c));
  *n = c;
  return MV_OK;
}

int mv_engine_create(int32_t device, const mv_problem_desc* pd, const mv_model_desc* md,
                     mv_engine** out) {
  if (!pd || !out) return fail(MV_ERR_ARG, "null argument");
  *out = nullptr;
  const int D = pd->D, V = pd->V, Dm = pd->Dm, C = pd->C;
  if (D <= 0 || V <= 0 || Dm <= 0 || C < 0) return fail(MV_ERR_ARG, "bad problem sizes");
  if (pd->D * 4 * 8 > 160 * 1024) return fail(MV_ERR_ARG, "D too large");
  if (md && (md->n_layers < 2 || md->n_layers > MAX_LAYERS))
    return fail(MV_ERR_ARG, "classifier must have 2..6 Dense layers");
  if (md) {
    if (md->dims[0] != D) return fail(MV_ERR_ARG, "model input width != D");
    for (int l = 1; l < md->n_layers; ++l)
      if (md->dims[l] % 16 != 0 || md->dims[l] > 512 || md->dims[l] <= 0)
        return fail(MV_ERR_ARG, "hidden widths must be multiples of 16 and <= 512");
    if (md->dims[md->n_layers] < 2 || md->dims[md->n_layers] > 8)
      return fail(MV_ERR_ARG, "softmax output width must be 2..8");
  }
  for (int j = 1; j < Dm; ++j)
    if (pd->mut_feats[j] <= pd->mut_feats[j - 1]) return fail(MV_ERR_ARG, "mut_feats not ascending");
  int ns[2] = {0, 0};
  for (int g = 0; g < V; ++g) {
    const int k = pd->gene_kind[g];
    if (k < 0 || k > 2) return fail(MV_ERR_ARG, "bad gene kind");
    const int sub = ns[k == MV_GENE_REAL ? 0 : 1]++;
    if (pd->gene_feat[g] < 0 || pd->gene_feat[g] > 0x7FFF || sub > 0x7FFF)
      return fail(MV_ERR_ARG, "feature/gene index too large for the packed gene table");
  }
  if (V > VARY_MAX_V || ((Dm + 15) & ~15) > VARY_MAX_V)
    return fail(MV_ERR_ARG, "genetic length / mutable features must be <= 1024");
  HIPCHK(hipSetDevice(device));
  mv_engine* e = new mv_engine();
  e->device = device;
  HostProblem& h = e->hp;
  h.D = D;
  h.V = V;
  h.Dm = Dm;
  h.C = C;
  h.n_ohe = pd->n_ohe;
  h.n_pool = pd->n_pool;
  h.norm = pd->norm;
  h.scale_obj = pd->scale_objectives;
  h.tol = pd->tol;
  h.kind.assign(pd->gene_kind, pd->gene_kind + V);
  h.feat.assign(pd->gene_feat, pd->gene_feat + V);
  h.ohe_off.assign(pd->n_ohe + 1, 0);
  if (pd->n_ohe > 0) std::memcpy(h.ohe_off.data(), pd->ohe_offsets, (pd->n_ohe + 1) * sizeof(int));
  const int n_ohe_feats = pd->n_ohe > 0 ? pd->ohe_offsets[pd->n_ohe] : 0;
  h.ohe_feats.assign(pd->ohe_feats, pd->ohe_feats + n_ohe_feats);
  h.mut.assign(pd->mut_feats, pd->mut_feats + Dm);
  h.op_code.assign(pd->op_code, pd->op_code + C);
  h.op_arg.assign(pd->op_arg, pd->op_arg + (size_t)C * 4);
  h.op_k.assign(pd->op_karg, pd->op_karg + (size_t)C * 2);
  h.pool.assign(pd->idx_pool, pd->idx_pool + pd->n_pool);
  h.mls.assign(D, 1.0);
  h.mlm.assign(D, 0.0);
  if (pd->ml_scale) std::memcpy(h.mls.data(), pd->ml_scale, D * sizeof(double));
  if (pd->ml_min) std::memcpy(h.mlm.data(), pd->ml_min, D * sizeof(double));
  if (md) {
    e->has_model = true;
    HostModel& m = e->hm;
    m.n_layers = md->n_layers;
    for (int l = 0; l <= md->n_layers; ++l) m.dims[l] = md->dims[l];
    for (int l = 0; l < md->n_layers; ++l) {
      m.W[l].assign(md->W[l], md->W[l] + (size_t)md->dims[l] * md->dims[l + 1]);
      m.b[l].assign(md->b[l], md->b[l] + md->dims[l + 1]);
    }
  }
  const int rc = build_problem(h, md ? &e->hm : nullptr, {}, e->p, e->prob_allocs);
  if (rc != MV_OK) {
    delete e;
    return rc;
  }
  // layer-1 bias fold of k_setup_states: the full W0 (feature rows) and b1
  hipError_t err = hipSuccess;
  auto K = [&](auto** dst, const auto* host, size_t n) {
    if (err == hipSuccess) err = e->keep(e->prob_allocs, dst, host, n);
  };
  if (md) {
    e->H1 = md->dims[1];
    K(&e->W1full, md->W[0], (size_t)D * e->H1);
    K(&e->b1, md->b[0], e->H1);
    e->p.bias[0] = e->b1;
  } else {
    e->H1 = 16;
    std::vector<float> zero(16, 0.f);
    K(&e->W1full, zero.data(), 16);
    K(&e->b1, zero.data(), 16);
  }
  if (err != hipSuccess) {
    delete e;
    return fail(MV_ERR_HIP, std::string("upload: ") + hipGetErrorString(err));
  }
  *out = e;
  return MV_OK;
}

void mv_engine_destroy(mv_engine* e) { delete e; }

// attack: the attack's layout (compact when mv_set_states found fixed genes)
static RowsArgs base_rows(const mv_engine* e, bool attack = false);

// The genes no attack on this state set can change: integer genes (not one-hot) whose
// bounds are equal and whose initial value -- x_init, already integral -- is that bound in
// every state (crossover swaps equal values, a mutation is clamped back to the bound).  Such
// genes exist only in IDENT problems here (botnet: 120 of 432); MV_COMPACT=0 keeps them all.
// Returns the genes to store (ascending), or empty when every gene is stored.
static bool compact_allowed(const mv_engine* e) {
  const char* env = std::getenv("MV_COMPACT");
  return !(env && env[0] == '0') && e->p.ident && e->has_model;
}

// Gene g can never change in state b (the compact layout's rule, above).
static bool gene_fixed(const HostProblem& h, int g, const double* x_init, const double* xl,
                       const double* xu, int b) {
  if (h.kind[g] != MV_GENE_INT) return false;
  const int f = h.feat[g];
  const double x = x_init[(size_t)b * h.D + f], lo = xl[(size_t)b * h.D + f],
               hi = xu[(size_t)b * h.D + f];
  return lo == hi && x == lo && std::rint(x) == x;
}

static std::vector<int> stored_genes(const mv_engine* e, int B, const double* x_init,
                                     const double* xl, const double* xu) {
  const HostProblem& h = e->hp;
  std::vector<int> keep;
  if (!compact_allowed(e)) return keep;
  for (int g = 0; g < h.V; ++g) {
    bool fixed = true;
    for (int b = 0; b < B && fixed; ++b) fixed = gene_fixed(h, g, x_init, xl, xu, b);
    if (!fixed) keep.push_back(g);
  }
  if ((int)keep.size() == h.V || keep.empty()) keep.clear();
  return keep;
}

static hipError_t alloc_states(mv_engine* e, const DProblem& p, int B, const double* x_init,
                               std::vector<void*>& list, DStates& s, double*& genes0) {
  s = DStates{};
  s.B = B;
  hipError_t err = hipSuccess;
  auto K = [&](auto** dst, const auto* host, size_t n) {
    if (err == hipSuccess) err = e->keep(list, dst, host, n);
  };
  K((double**)&s.x_init, x_init, (size_t)B * p.D);
  K((double**)&s.gl, (const double*)nullptr, (size_t)B * p.V);
  K((double**)&s.gu, (const double*)nullptr, (size_t)B * p.V);
  K((unsigned char**)&s.sblob, (const unsigned char*)nullptr, (size_t)B * vary_offsets(p).sb);
  K((float**)&s.bias1, (const float*)nullptr, (size_t)B * e->H1);
  K(&genes0, (const double*)nullptr, (size_t)B * p.V);
  return err;
}

int mv_set_states(mv_engine* e, int32_t B, const double* x_init, const double* xl,
                  const double* xu, const int32_t* minimize_class, void* stream) {
  if (!e || B <= 0 || !x_init || !xl || !xu || !minimize_class)
    return fail(MV_ERR_ARG, "bad mv_set_states arguments");
  HIPCHK(hipSetDevice(e->device));
  // a model-less engine (host classifier plugin) evaluates f2 / f3 only: no class check
  const int nout = e->has_model ? e->p.dims[e->p.n_layers] : INT32_MAX;
  for (int b = 0; b < B; ++b)
    if (minimize_class[b] < 0 || minimize_class[b] >= nout)
      return fail(MV_ERR_ARG, "minimize_class out of range");
  // the attack's compact layout, when this state set has genes that never change (or the
  // layout mv_set_gene_layout requested, checked against this batch before anything bound is
  // released; the request applies to this call only)
  std::vector<int> keep;
  if (e->layout_req.empty()) {
    keep = stored_genes(e, B, x_init, xl, xu);
  } else {
    const std::vector<int> req = std::move(e->layout_req);
    e->layout_req.clear();
    if (compact_allowed(e)) {
      size_t j = 0;
      for (int g = 0; g < e->hp.V; ++g) {
        if (j < req.size() && req[j] == g) {
          ++j;
          continue;
        }
        for (int b = 0; b < B; ++b)
          if (!gene_fixed(e->hp, g, x_init, xl, xu, b))
            return fail(MV_ERR_ARG, "mv_set_gene_layout: gene " + std::to_string(g) +
                                        " is not fixed in bound state " + std::to_string(b));
      }
      keep = req;
      if ((int)keep.size() == e->hp.V) keep.clear();
    }
  }
  HIPCHK(hipDeviceSynchronize());
  e->free_list(e->cstate_allocs);
  e->free_list(e->state_allocs);
  e->free_list(e->attack_allocs);
  e->d_phase = nullptr;
  e->front_scr = nullptr;
  e->off_scr = nullptr;
  e->attack_ready = false;
  e->compact = false;
  e->B = 0;
  double *dxl = nullptr, *dxu = nullptr;
  hipError_t err = alloc_states(e, e->p, B, x_init, e->state_allocs, e->s, e->genes0);
  if (err == hipSuccess) err = e->keep(e->state_allocs, &dxl, xl, (size_t)B * e->p.D);
  if (err == hipSuccess) err = e->keep(e->state_allocs, &dxu, xu, (size_t)B * e->p.D);
  if (err == hipSuccess)
    err = e->keep(e->state_allocs, (int**)&e->s.min_class, minimize_class, (size_t)B);
  if (err != hipSuccess) return fail(MV_ERR_HIP, std::string("alloc: ") + hipGetErrorString(err));
  int slot = 0;
  HIPCHK(stage_rows(base_rows(e), (hipStream_t)stream, &slot));
  HIPCHK(launch_setup_states(slot, B, e->s.x_init, dxl, dxu, e->W1full, e->b1, (double*)e->s.gl,
                             (double*)e->s.gu, (unsigned char*)e->s.sblob, (float*)e->s.bias1,
                             e->genes0, (hipStream_t)stream));
  HIPCHK(release_rows(slot, (hipStream_t)stream));
  if (!keep.empty()) {
    if (keep != e->stored) {
      HIPCHK(hipDeviceSynchronize());
      e->free_list(e->compact_allocs);
      e->stored.clear();
      const int rc = build_problem(e->hp, e->has_model ? &e->hm : nullptr, keep, e->pc,
                                   e->compact_allocs);
      if (rc != MV_OK) return rc;
      e->pc.bias[0] = e->b1;
      e->stored = keep;
    }
    err = alloc_states(e, e->pc, B, x_init, e->cstate_allocs, e->sc, e->genes0c);
    if (err != hipSuccess) return fail(MV_ERR_HIP, std::string("alloc: ") + hipGetErrorString(err));
    e->sc.min_class = e->s.min_class;
    e->compact = true;
    HIPCHK(stage_rows(base_rows(e, true), (hipStream_t)stream, &slot));
    HIPCHK(launch_setup_states(slot, B, e->sc.x_init, dxl, dxu, e->W1full, e->b1,
                               (double*)e->sc.gl, (double*)e->sc.gu, (unsigned char*)e->sc.sblob,
                               (float*)e->sc.bias1, e->genes0c, (hipStream_t)stream));
    HIPCHK(release_rows(slot, (hipStream_t)stream));
  }
  e->B = B;
  return MV_OK;
}

static RowsArgs base_rows(const mv_engine* e, bool attack) {
  RowsArgs a{};
  a.p = attack ? e->ap() : e->p;
  a.s = attack ? e->as() : e->s;
  a.eta = 20.0;
  a.cx_prob = e->cx_prob;
  a.cx_kind = e->cx_kind;
  a.sbx_eta = e->sbx_eta;
  a.state_keys = e->state_keys;
  a.key0 = e->key0;
  a.do_eval = 1;
  a.states_all = e->B;
  a.p.mlp_bf16 = e->has_model && e->mlp_bf16;
  return a;
}

int mv_evaluate(mv_engine* e, int32_t n, const double* genes, double* F, double* G, void* stream) {
  if (!e || n <= 0 || !genes || !F) return fail(MV_ERR_ARG, "bad mv_evaluate arguments");
  if (e->B <= 0) return fail(MV_ERR_STATE, "no states bound (mv_set_states)");
  if (!on_device(genes, e->device) || !on_device(F, e->device) || !on_device(G, e->device))
    return fail(MV_ERR_ARG, "mv_evaluate: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  RowsArgs a = base_rows(e);
  a.n = n;
  a.total = e->B * n;
  a.mode = 0;
  a.genes_in = genes;
  a.in_rows = n;
  a.out_rows = n;
  a.F = F;
  a.G = G;
  HIPCHK(e->ensure_xml((size_t)a.total));
  a.xml = e->xml;
  int slot = 0;
  HIPCHK(stage_rows(a, (hipStream_t)stream, &slot));
  HIPCHK(launch_rows(a, slot, 0, 0, (hipStream_t)stream));
  HIPCHK(release_rows(slot, (hipStream_t)stream));
  return MV_OK;
}

int mv_decode(mv_engine* e, int32_t n, const double* genes, double* x, void* stream) {
  if (!e || n < 0 || (n > 0 && (!genes || !x))) return fail(MV_ERR_ARG, "bad mv_decode arguments");
  if (e->B <= 0) return fail(MV_ERR_STATE, "no states bound (mv_set_states)");
  if (!on_device(genes, e->device) || !on_device(x, e->device))
    return fail(MV_ERR_ARG, "mv_decode: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(launch_decode(e->p, e->s, e->B, n, genes, x, (hipStream_t)stream));
  return MV_OK;
}

int mv_constraints(mv_engine* e, int32_t n, const double* x, double* G, void* stream) {
  if (!e || n < 0 || (n > 0 && (!x || !G))) return fail(MV_ERR_ARG, "bad mv_constraints arguments");
  if (!on_device(x, e->device) || !on_device(G, e->device))
    return fail(MV_ERR_ARG, "mv_constraints: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  int slot = 0;
  HIPCHK(stage_rows(base_rows(e), (hipStream_t)stream, &slot));
  HIPCHK(launch_constraints(e->p, slot, n, x, G, (hipStream_t)stream));
  HIPCHK(release_rows(slot, (hipStream_t)stream));
  return MV_OK;
}

int mv_variation(mv_engine* e, int32_t P, int32_t O, uint64_t seed, int32_t gen, const double* pop,
                 const int32_t* parents, double* off, void* stream) {
  if (!e || P <= 1 || O <= 0 || (O & 1) || !pop || !parents || !off)
    return fail(MV_ERR_ARG, "bad mv_variation arguments (O must be even)");
  if (e->B <= 0) return fail(MV_ERR_STATE, "no states bound (mv_set_states)");
  if (!on_device(pop, e->device) || !on_device(parents, e->device) || !on_device(off, e->device))
    return fail(MV_ERR_ARG, "mv_variation: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  RowsArgs a = base_rows(e);
  a.n = O;
  a.total = e->B * O;
  a.mode = 1;
  a.genes_in = pop;
  a.in_rows = P;
  a.parents = parents;
  a.genes_out = off;
  a.out_rows = O;
  a.seed = seed;
  a.do_eval = 0;
  int slot = 0;
  HIPCHK(stage_rows(a, (hipStream_t)stream, &slot));
  HIPCHK(launch_vary(a, slot, gen, 0, (hipStream_t)stream));
  HIPCHK(release_rows(slot, (hipStream_t)stream));
  return MV_OK;
}

int mv_survive(int32_t B, int32_t N, int32_t n_survive, const double* F, int32_t R,
               const double* ref_points, double mu, uint64_t seed, int32_t gen, double* ideal,
               double* worst, double* extreme, int32_t* has_extreme, int32_t* survivors,
               int32_t* rank, int32_t* order, int32_t* n_ranked, int32_t* niche, double* dist,
               double* nadir, void* stream) {
  if (B <= 0 || N <= 0 || N > SURV_NMAX || R <= 0 || R > SURV_RMAX || n_survive <= 0 ||
      n_survive > N || !F || !ref_points || !ideal || !worst || !extreme || !has_extreme ||
      !survivors)
    return fail(MV_ERR_ARG, "bad mv_survive arguments (N <= 1024, R <= 640, n_survive <= N)");
  if (surv_lds_bytes(N, R, 1) > 160 * 1024)
    return fail(MV_ERR_ARG, "mv_survive: N and R too large for the survival LDS workspace");
  {  // no engine here: every buffer must live on the current device
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    const void* bufs[] = {F, ref_points, ideal, worst, extreme, has_extreme, survivors, rank,
                          order, n_ranked, niche, dist, nadir};
    for (const void* q : bufs)
      if (!on_device(q, dev))
        return fail(MV_ERR_ARG, "mv_survive: a buffer lives on another device than the current one");
  }
  SurvArgs a{};
  a.N = N;
  a.n_survive = n_survive;
  a.F = F;
  a.ref = ref_points;
  a.R = R;
  a.mu = mu;
  a.seed = seed;
  a.gen = gen;
  a.ideal = ideal;
  a.worst = worst;
  a.extreme = extreme;
  a.has_extreme = has_extreme;
  a.survivors = survivors;
  a.rank = rank;
  a.order = order;
  a.n_ranked = n_ranked;
  a.niche = niche;
  a.dist = dist;
  a.nadir = nadir;
  if (N > SURV_NLDS) {  // dominance bitsets in HBM, stream-ordered scratch
    a.dom_stride = (size_t)N * ((N + 63) / 64);
    HIPCHK(hipMallocAsync((void**)&a.dom_g, (size_t)B * a.dom_stride * 8, (hipStream_t)stream));
  }
  const hipError_t le = launch_survive(a, B, (hipStream_t)stream);
  if (a.dom_g) HIPCHK(hipFreeAsync(a.dom_g, (hipStream_t)stream));
  HIPCHK(le);
  return MV_OK;
}

int mv_select_parents(int32_t B, int32_t P, int32_t O, uint64_t seed, int32_t gen,
                      int32_t* parents, void* stream) {
  if (B <= 0 || P <= 1 || O <= 0 || !parents) return fail(MV_ERR_ARG, "bad mv_select_parents");
  const int n_m = (O + 1) / 2, slots = ((n_m * 4 + P - 1) / P) * P;
  int p2 = 1;
  while (p2 < slots) p2 <<= 1;
  if (P > 8192 || (size_t)p2 * 8 + (size_t)slots * 4 > 160 * 1024)
    return fail(MV_ERR_ARG, "mv_select_parents: population or offspring count too large");
  {
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (!on_device(parents, dev))
      return fail(MV_ERR_ARG, "mv_select_parents: parents live on another device than the current one");
  }
  HIPCHK(launch_select(B, P, O, seed, 0u, gen, nullptr, parents, (hipStream_t)stream));
  return MV_OK;
}

int mv_set_profiling(mv_engine* e, int32_t enabled) {
  if (!e) return fail(MV_ERR_ARG, "null engine");
  e->profiling = enabled != 0;
  return MV_OK;
}

static int ensure_events(std::vector<hipEvent_t>& v, size_t n) {
  while (v.size() < n) {
    hipEvent_t ev;
    HIPCHK(hipEventCreate(&ev));
    v.push_back(ev);
  }
  return MV_OK;
}

int mv_attack_run(mv_engine* e, const mv_attack_params* prm, void* stream_) {
  if (!e || !prm) return fail(MV_ERR_ARG, "null argument");
  if (!e->has_model)
    return fail(MV_ERR_STATE, "mv_attack_run needs a device classifier (hosted plugins run "
                              "the generation loop from the host)");
  if (e->B <= 0) return fail(MV_ERR_STATE, "no states bound (mv_set_states)");
  const int P = prm->pop_size, O = prm->n_offsprings, G = prm->n_gen, R = prm->n_ref;
  if (P < 2 || O < 2 || (O & 1) || G < 1 || R < 1 || R > SURV_RMAX || P + O > SURV_NMAX ||
      !prm->ref_points || prm->history < 0 || prm->history > 2)
    return fail(MV_ERR_ARG,
                "bad attack parameters (even n_offsprings, pop_size + n_offsprings <= 1024, "
                "n_ref <= 640)");
  {
    const int n_m = (O + 1) / 2, pslots = ((n_m * 4 + P - 1) / P) * P;
    const int ptab = plan_tab_words(e->ap().Vr, e->ap().V);
    if (surv_lds_bytes(P + O, R, pslots, ptab, P + O > SURV_NLDS ? SURV_T_BIG : SURV_T_MID) >
            160 * 1024 ||
        surv_lds_bytes(P, R, pslots, ptab, P > SURV_NLDS ? SURV_T_BIG : SURV_T_MID) > 160 * 1024)
      return fail(MV_ERR_ARG, "pop_size + n_offsprings and n_ref too large for the survival LDS");
  }
  hipStream_t stream = (hipStream_t)stream_;
  HIPCHK(hipSetDevice(e->device));
  const DProblem& ap = e->ap();  // the attack's layout (compact: fixed genes not stored)
  const int B = e->B, V = ap.V, S = P + O;
  const int hist_w = prm->history == 2 ? 3 + ap.C : 3;
  const int hist_rows = P + (G - 1) * O;
  // the offspring rows' kernel: k_genc reads a variation plan written by k_survive
  bool use_plan = false;
  {
    RowsArgs t = base_rows(e, true);
    t.n = O;
    t.total = B * O;
    t.mode = 1;
    use_plan = row_kernel_kind(t) == 2;
  }
  const bool realloc = !e->attack_ready || e->P != P || e->O != O || e->R != R ||
                       e->hist_mode != prm->history || (prm->history && e->n_gen != G) ||
                       e->has_plan != use_plan;  // the budget sizes the history only
  if (realloc) {
    HIPCHK(hipDeviceSynchronize());
    e->free_list(e->attack_allocs);
    e->d_phase = nullptr;
      hipError_t err = hipSuccess;
    auto A = [&](auto** dst, size_t n) {
      if (err != hipSuccess) return;
      err = dalloc(dst, n);
      if (err == hipSuccess) e->attack_allocs.push_back((void*)*dst);
    };
    e->d_gphase = nullptr;
    e->gphase_n = 0;
    e->front_scr = nullptr;
    e->off_scr = nullptr;
    A(&e->pool, (size_t)B * S * V);
    A(&e->poolF, (size_t)B * S * 3);
    A(&e->pop_slot, (size_t)B * P);
    A(&e->free_slot, (size_t)B * O);
    A(&e->parents, (size_t)B * O);
    e->plan_hdr = nullptr;
    e->plan_mw = nullptr;
    e->plan_mu = nullptr;
    if (use_plan) {
      A(&e->plan_hdr, (size_t)B * O);
      A(&e->plan_mw, (size_t)B * O * PLAN_MUT);
      A(&e->plan_mu, (size_t)B * O * PLAN_MUT);
    }
    e->has_plan = use_plan;
    e->dom_g = nullptr;
    e->dom_stride = 0;
    if (S > SURV_NLDS) {
      e->dom_stride = (size_t)S * ((S + 63) / 64);
      A(&e->dom_g, (size_t)B * e->dom_stride);
    }
    A(&e->ideal, (size_t)B * 3);
    A(&e->worst, (size_t)B * 3);
    A(&e->extreme, (size_t)B * 9);
    A(&e->has_ext, (size_t)B);
    A(&e->ref, (size_t)R * 3);
    if (prm->history) A(&e->hist, (size_t)B * hist_rows * hist_w);
    if (err != hipSuccess)
      return fail(MV_ERR_HIP, std::string("attack alloc: ") + hipGetErrorString(err));
    e->P = P;
    e->O = O;
    e->S = S;
    e->R = R;
    e->n_gen = G;
    e->hist_mode = prm->history;
    e->hist_w = hist_w;
    e->hist_rows = hist_rows;
    e->attack_ready = true;
  }
  // Reference points: a previous attack still queued on another stream may read e->ref,
  // so they are re-uploaded only when they change, and then behind a device-wide sync.
  // (Callers pass the same energy directions every time; the common case copies nothing
  // and keeps the host running ahead of the GPU.)
  if (realloc || e->ref_host.size() != (size_t)R * 3 ||
      std::memcmp(e->ref_host.data(), prm->ref_points, (size_t)R * 3 * sizeof(double)) != 0) {
    HIPCHK(hipDeviceSynchronize());
    e->ref_host.assign(prm->ref_points, prm->ref_points + (size_t)R * 3);
    HIPCHK(hipMemcpy(e->ref, e->ref_host.data(), (size_t)R * 3 * sizeof(double),
                     hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL(k_fill_d, dim3(64), dim3(256), 0, stream, e->ideal, (size_t)B * 3,
                     (double)INFINITY);
  hipLaunchKernelGGL(k_fill_d, dim3(64), dim3(256), 0, stream, e->worst, (size_t)B * 3,
                     (double)-INFINITY);
  hipLaunchKernelGGL(k_fill_i, dim3(64), dim3(256), 0, stream, e->has_ext, (size_t)B, 0);
  HIPCHK(hipGetLastError());
  HIPCHK(launch_init_pool(B, P, O, V, S, e->ag0(), e->pool, e->pop_slot, e->free_slot, stream));
  HIPCHK(e->ensure_xml((size_t)B * (P > O ? P : O)));
  // Initial states are independent: split them into state groups, each running its own
  // generation chain on its own stream, so one group's latency-bound survival overlaps the
  // other groups' throughput-bound kernels.  Results do not depend on the grouping (every
  // draw is keyed by the row inside its state).  Profiling runs use one group so the
  // per-kernel event times are those of the kernels alone.
  int ngrp = B / 64;  // about 100 states per group at the botnet size; at most 4 =
                      // GPU_MAX_HW_QUEUES (round 5: MV_GROUPS 6 / 8, with GPU_MAX_HW_QUEUES
                      // 6 / 8: 148 / 147 vs 218 M evals/s; round 2: 35 % slower)
  ngrp = ngrp > 4 ? 4 : ngrp;
  if (const char* g = std::getenv("MV_GROUPS")) ngrp = std::atoi(g);
  if (e->profiling) ngrp = 1;
  ngrp = ngrp < 1 ? 1 : (ngrp > MAX_GROUPS ? MAX_GROUPS : (ngrp > B ? B : ngrp));
  HIPCHK(e->ensure_streams(ngrp));
  hipStream_t gs[MAX_GROUPS];
  int gb0[MAX_GROUPS + 1];
  for (int q = 0; q <= ngrp; ++q) gb0[q] = (int)((long long)B * q / ngrp);
  gs[0] = stream;
  if (ngrp > 1) HIPCHK(hipEventRecord(e->ev_fork, stream));
  for (int q = 1; q < ngrp; ++q) {
    gs[q] = e->streams[q];
    HIPCHK(hipStreamWaitEvent(gs[q], e->ev_fork, 0));
  }
  const int H1 = e->H1, D = ap.D;
  const unsigned sbb = vary_offsets(ap).sb;
  const size_t Dm4 = ap.Dm4;
  auto group_rows = [&](RowsArgs r, int q, int n_per_state) {
    const size_t b0 = gb0[q];
    r.s.B = gb0[q + 1] - gb0[q];
    r.s.x_init += b0 * D;
    r.s.gl += b0 * V;
    r.s.gu += b0 * V;
    r.s.sblob += b0 * sbb;
    r.s.bias1 += b0 * H1;
    r.s.min_class += b0;
    r.total = r.s.B * n_per_state;
    r.key0 += (uint32_t)b0;  // per-state streams: the group's first state
    if (r.genes_in) r.genes_in += b0 * r.in_rows * V;
    if (r.genes_out) r.genes_out += b0 * r.out_rows * V;
    if (r.parents) r.parents += b0 * O;
    if (r.out_map) r.out_map += b0 * r.n;
    if (r.plan_hdr) {
      r.plan_hdr += b0 * O;
      r.plan_mw += b0 * O * PLAN_MUT;
      r.plan_mu += b0 * O * PLAN_MUT;
    }
    if (r.F) r.F += b0 * r.out_rows * 3;
    if (r.hist) r.hist += b0 * (size_t)r.hist_rows * r.hist_w;
    // Each group owns xml rows [b0, b1) x max(P, O): one group's initial evaluation (n = P)
    // may still be reading its rows while a faster group already writes its first
    // offspring (n = O), so the regions must not depend on the phase's n.
    r.xml += b0 * (size_t)(P > O ? P : O) * Dm4;
    return r;
  };
  auto group_surv = [&](SurvArgs s, int q) {
    const size_t b0 = gb0[q];
    s.F += b0 * S * 3;
    s.pop_slot += b0 * P;
    s.free_slot += b0 * O;
    s.pop_slot_out += b0 * P;
    s.ideal += b0 * 3;
    s.worst += b0 * 3;
    s.extreme += b0 * 9;
    s.has_extreme += b0;
    s.key0 += (uint32_t)b0;
    if (s.parents_out) s.parents_out += b0 * O;
    if (s.phase) s.phase += b0 * 32;
    if (s.dom_g) s.dom_g += b0 * s.dom_stride;
    if (s.plan_hdr) {
      s.plan_hdr += b0 * O;
      s.plan_mw += b0 * O * PLAN_MUT;
      s.plan_mu += b0 * O * PLAN_MUT;
    }
    return s;
  };
  // initial population evaluation (pymoo _initialize)
  RowsArgs ev = base_rows(e, true);
  ev.n = P;
  ev.mode = 0;
  ev.genes_in = e->pool;
  ev.in_rows = S;
  ev.out_rows = S;
  ev.F = e->poolF;
  ev.hist = prm->history ? e->hist : nullptr;
  ev.hist_rows = hist_rows;
  ev.hist_w = hist_w;
  ev.xml = e->xml;
  SurvArgs sa{};
  sa.n_survive = P;
  sa.P = P;
  sa.O = O;
  sa.F = e->poolF;
  sa.S = S;
  sa.pop_slot = e->pop_slot;
  sa.free_slot = e->free_slot;
  sa.pop_slot_out = e->pop_slot;
  sa.ref = e->ref;
  sa.R = R;
  sa.mu = prm->mu;
  sa.seed = prm->seed;
  sa.state_keys = e->state_keys;
  sa.key0 = e->key0;
  sa.ideal = e->ideal;
  sa.worst = e->worst;
  sa.extreme = e->extreme;
  sa.has_extreme = e->has_ext;
  sa.O_next = O;
  sa.dom_g = e->dom_g;
  sa.dom_stride = e->dom_stride;
  {  // 10-wave survival workgroups when every state fits two workgroups per CU (SurvArgs.wide)
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 0;
    (void)hipGetLastError();
    // 2: small attacks (every state has half a CU or more to itself -- configs[0], the
    // per-GPU share of 8-GPU strong scaling): 16-wave workgroups, so one state's issue-
    // and latency-bound phases interleave four waves per SIMD
    sa.wide = 2 * B <= cus ? 2 : B <= 2 * cus ? 1 : 0;
    if (const char* w = std::getenv("MV_SURV_WIDE")) sa.wide = std::atoi(w);  // A/B
  }
  if (use_plan) {
    const VaryOff vo = vary_offsets(ap);
    sa.plan_hdr = e->plan_hdr;
    sa.plan_mw = e->plan_mw;
    sa.plan_mu = e->plan_mu;
    sa.geo = (const uint32_t*)(ap.vblob + vo.geo);
    sa.cmap = (const int*)(ap.vblob + vo.cmap);
    sa.ginfo = (const int*)(ap.vblob + vo.ginfo);
    sa.Vr = ap.Vr;
    sa.V = ap.V;
    sa.n_sub0 = ap.n_sub[0];
    sa.n_sub1 = ap.n_sub[1];
    sa.cx_prob = e->cx_prob;
    sa.cx_sbx = e->cx_kind == 1;
  }
  if (std::getenv("MV_SURV_PHASES")) {
    if (!e->d_phase) {
      HIPCHK(hipMalloc((void**)&e->d_phase, (size_t)B * 32 * sizeof(long long)));
      e->attack_allocs.push_back(e->d_phase);
    }
    sa.phase = e->d_phase;
  }
  // dummy survival at initialisation: n_survive == len(pop)
  sa.N = P;
  sa.gen = 0;
  sa.parents_out = G > 1 ? e->parents : nullptr;
  sa.sel_gen = 1;
  for (int q = 0; q < ngrp; ++q) {
    int slot_ev = 0;
    const RowsArgs evq = group_rows(ev, q, P);
    HIPCHK(stage_rows(evq, gs[q], &slot_ev));
    HIPCHK(launch_rows(evq, slot_ev, 0, 0, gs[q]));
    HIPCHK(release_rows(slot_ev, gs[q]));
    HIPCHK(launch_survive(group_surv(sa, q), gb0[q + 1] - gb0[q], gs[q]));
  }
  if (e->profiling) {
    if (ensure_events(e->ev_var, 2 * (size_t)G) != MV_OK) return MV_ERR_HIP;
    if (ensure_events(e->ev_mlp, (size_t)G) != MV_OK) return MV_ERR_HIP;
    if (ensure_events(e->ev_cons, (size_t)G) != MV_OK) return MV_ERR_HIP;
    if (ensure_events(e->ev_surv, 2 * (size_t)G) != MV_OK) return MV_ERR_HIP;
    if (ensure_events(e->ev_kx, 6 * (size_t)G) != MV_OK) return MV_ERR_HIP;
  }
  e->n_var_rec = 0;
  e->n_surv_rec = 0;
  RowsArgs va = base_rows(e, true);
  va.n = O;
  va.mode = 1;
  va.genes_in = e->pool;
  va.in_rows = S;
  va.parents = e->parents;
  va.genes_out = e->pool;
  va.out_rows = S;
  va.out_map = e->free_slot;
  va.F = e->poolF;
  va.hist = prm->history ? e->hist : nullptr;
  va.hist_rows = hist_rows;
  va.hist_w = hist_w;
  va.seed = prm->seed;
  va.xml = e->xml;
  if (use_plan) {
    va.plan_hdr = e->plan_hdr;
    va.plan_mw = e->plan_mw;
    va.plan_mu = e->plan_mu;
  }
  const bool mlp_ph = std::getenv("MV_MLP_PHASES") != nullptr;
  if ((std::getenv("MV_GEN_PHASES") || mlp_ph) && ngrp == 1) {  // development: phase clocks
    const size_t n = (size_t)B * O * 16;  // >= grid * 16 (at least one row per workgroup)
    if (e->gphase_n < n) {
      HIPCHK(hipMalloc((void**)&e->d_gphase, n * sizeof(long long)));
      e->attack_allocs.push_back(e->d_gphase);
      e->gphase_n = n;
    }
    HIPCHK(hipMemsetAsync(e->d_gphase, 0, n * sizeof(long long), stream));
    (mlp_ph ? va.mphase : va.gphase) = e->d_gphase;
    e->gphase_mlp = mlp_ph;
  }
  int slot_va[MAX_GROUPS];
  RowsArgs vq[MAX_GROUPS];
  for (int q = 0; q < ngrp; ++q) {
    vq[q] = group_rows(va, q, O);
    HIPCHK(stage_rows(vq[q], gs[q], &slot_va[q]));
  }
  sa.N = P + O;
  for (int g = 1; g < G; ++g) {
    const int hist_row0 = P + (g - 1) * O;
    sa.gen = g;
    sa.parents_out = g + 1 < G ? e->parents : nullptr;
    sa.sel_gen = g + 1;
    for (int q = 0; q < ngrp; ++q) {
      hipStream_t st = gs[q];
      const bool prof = e->profiling && q == 0;
      // profiled steps: each launch takes an armed event pair (kernel-exact stamps); a step
      // that launches no kernel (k_genc's empty k_cons) records the pair back to back
      struct Disarm {
        ~Disarm() { g_ev_start = g_ev_stop = nullptr; }
      } disarm;
      auto arm = [&](hipEvent_t a0, hipEvent_t a1) {
        g_ev_start = a0;
        g_ev_stop = a1;
      };
      auto settle = [&]() -> hipError_t {
        if (!g_ev_start) return hipSuccess;
        hipError_t r = hipEventRecord(g_ev_start, st);
        if (r == hipSuccess) r = hipEventRecord(g_ev_stop, st);
        g_ev_start = g_ev_stop = nullptr;
        return r;
      };
      hipEvent_t* kx = prof ? &e->ev_kx[6 * (size_t)e->n_var_rec] : nullptr;
      if (prof) arm(kx[0], kx[1]);
      HIPCHK(launch_gen(vq[q], slot_va[q], g, hist_row0, st));
      if (prof) HIPCHK(settle());
      if (prof) arm(kx[2], kx[3]);
      HIPCHK(launch_cons(vq[q], slot_va[q], hist_row0, st));
      if (prof) HIPCHK(settle());
      if (prof) arm(kx[4], kx[5]);
      HIPCHK(launch_mlp(vq[q], slot_va[q], hist_row0, st));
      if (prof) {
        HIPCHK(settle());
        ++e->n_var_rec;
        arm(e->ev_surv[2 * (size_t)e->n_surv_rec], e->ev_surv[2 * (size_t)e->n_surv_rec + 1]);
      }
      HIPCHK(launch_survive(group_surv(sa, q), gb0[q + 1] - gb0[q], st));
      if (prof) {
        HIPCHK(settle());
        ++e->n_surv_rec;
      }
    }
  }
  for (int q = 0; q < ngrp; ++q) HIPCHK(release_rows(slot_va[q], gs[q]));
  for (int q = 1; q < ngrp; ++q) {  // join: the caller's stream waits for every group
    HIPCHK(hipEventRecord(e->ev_join[q], gs[q]));
    HIPCHK(hipStreamWaitEvent(stream, e->ev_join[q], 0));
  }
  return MV_OK;
}

int mv_get_row_kernel(mv_engine* e, int32_t* kind) {
  if (!e || !kind) return fail(MV_ERR_ARG, "null argument");
  RowsArgs a = base_rows(e, true);
  a.n = 2;
  a.total = 2;
  a.mode = 1;
  *kind = row_kernel_kind(a);
  return MV_OK;
}

int mv_get_mlp_kernel(mv_engine* e, int32_t* kind) {
  if (!e || !kind) return fail(MV_ERR_ARG, "null argument");
  *kind = mlp_kernel_kind(base_rows(e, true).p);
  return MV_OK;
}

int mv_get_kernel_times(mv_engine* e, double* vary_ms, double* mlp_ms, double* survive_ms,
                        int32_t* n_generations) {
  if (!e) return fail(MV_ERR_ARG, "null engine");
  double tv = 0.0, tm = 0.0, ts = 0.0;
  for (int i = 0; i < e->n_var_rec; ++i) {  // kernel-exact pairs (ev_kx)
    float ms = 0.f, ms1 = 0.f, ms2 = 0.f;
    const hipEvent_t* kx = &e->ev_kx[6 * (size_t)i];
    HIPCHK(hipEventSynchronize(kx[5]));
    HIPCHK(hipEventElapsedTime(&ms, kx[0], kx[1]));
    HIPCHK(hipEventElapsedTime(&ms1, kx[2], kx[3]));
    HIPCHK(hipEventElapsedTime(&ms2, kx[4], kx[5]));
    tv += (double)ms + ms1;
    tm += ms2;
  }
  for (int i = 0; i < e->n_surv_rec; ++i) {
    float ms = 0.f;
    HIPCHK(hipEventSynchronize(e->ev_surv[2 * i + 1]));
    HIPCHK(hipEventElapsedTime(&ms, e->ev_surv[2 * i], e->ev_surv[2 * i + 1]));
    ts += ms;
  }
  if (vary_ms) *vary_ms = tv;
  if (mlp_ms) *mlp_ms = tm;
  if (survive_ms) *survive_ms = ts;
  if (n_generations) *n_generations = e->n_var_rec < e->n_surv_rec ? e->n_var_rec : e->n_surv_rec;
  if (e->d_gphase && e->gphase_n) {  // development aid: k_genc phase split, last generation
    std::vector<long long> g(e->gphase_n);
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(g.data(), e->d_gphase, g.size() * sizeof(long long), hipMemcpyDeviceToHost));
    double acc[6] = {0};
    long long w0 = INT64_MAX, w1 = 0;
    int n = 0;
    std::vector<double> dur;
    const size_t stride = e->gphase_mlp ? 16 : 8;
    double sub[4] = {0};
    for (size_t w = 0; w * stride + stride <= g.size(); ++w) {
      const long long* q = &g[w * stride];
      if (stride == 16 && q[8] && q[12])
        for (int k = 0; k < 4; ++k) sub[k] += (double)(q[9 + k] - q[8 + k]);
      if (!q[0] || !q[5]) continue;
      for (int k = 1; k <= 5; ++k) acc[k] += (double)(q[k] - q[k - 1]);
      w0 = std::min(w0, q[6]);
      w1 = std::max(w1, q[7]);
      dur.push_back((double)(q[7] - q[6]));
      ++n;
    }
    if (n) {
      std::sort(dur.begin(), dur.end());
      if (e->gphase_mlp)
        std::fprintf(stderr, "[mv] k_mlp phase cycles (mean over %d workgroups, first tile): "
                     "issue=%.0f chunk0=%.0f layer0=%.0f hidden=%.0f final=%.0f | workgroup "
                     "wall (100 MHz ticks) p50=%.0f max=%.0f, launch span=%lld | chunk 2: "
                     "loads=%.0f mfma=%.0f store=%.0f barrier=%.0f\n", n, acc[1] / n,
                     acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n, dur[dur.size() / 2],
                     dur.back(), w1 - w0, sub[0] / n, sub[1] / n, sub[2] / n, sub[3] / n);
      else
      std::fprintf(stderr, "[mv] k_genc phase cycles (mean over %d workgroups): stage1=%.0f draws=%.0f "
                   "rows1=%.0f stage2=%.0f rows2=%.0f | workgroup wall (100 MHz ticks) p50=%.0f "
                   "max=%.0f, launch span=%lld\n", n, acc[1] / n, acc[2] / n, acc[3] / n,
                   acc[4] / n, acc[5] / n, dur[dur.size() / 2], dur.back(), w1 - w0);
    }
  }
  if (e->d_phase && e->B > 0) {  // development aid: survival phase split of the last generation
    std::vector<long long> ph((size_t)e->B * 32);
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(ph.data(), e->d_phase, ph.size() * sizeof(long long), hipMemcpyDeviceToHost));
    double acc[32] = {0};
    for (int b = 0; b < e->B; ++b)
      for (int k = 1; k < 10; ++k) acc[k] += (double)(ph[(size_t)b * 32 + k] - ph[(size_t)b * 32 + k - 1]);
    std::fprintf(stderr, "[mv] survival phase cycles (mean over %d states):", e->B);
    for (int k = 1; k < 10; ++k) std::fprintf(stderr, " p%d=%.0f", k, acc[k] / e->B);
    // sub-phase marks (cycles since phase 0): 21/22 extremes (ASF loop, combine), 16..20
    // niching (keys, member lists, ranks, levels, round keys)
    std::fprintf(stderr, " | t:");
    for (int k : {3, 21, 22, 25, 26, 4, 5, 10, 6, 16, 17, 18, 19, 20, 7}) {
      double t = 0.0;
      for (int b = 0; b < e->B; ++b) t += (double)(ph[(size_t)b * 32 + k] - ph[(size_t)b * 32]);
      std::fprintf(stderr, " %d=%.0f", k, t / e->B);
    }
    double red = 0.0, afast = 0.0, nflag = 0.0;
    for (int b = 0; b < e->B; ++b) {
      const long long* q = &ph[(size_t)b * 32];
      red += (double)(q[11] - q[1]);
      afast += (double)(q[10] - q[5]);
      nflag += (double)q[12];
    }
    double tplan = 0.0, ttour = 0.0;
    for (int b = 0; b < e->B; ++b) {
      const long long* q = &ph[(size_t)b * 32];
      tplan += (double)(q[24] - q[23]);
    }
    std::fprintf(stderr, " | ideal/worst=%.0f assoc_fast=%.0f flagged=%.1f plan=%.0f", red / e->B,
                 afast / e->B, nflag / e->B, tplan / e->B);
    (void)ttour;
    // the launch lasts as long as its slowest state: per-phase maxima and the total's tail
    std::vector<double> tot(e->B);
    double pmax[10] = {0};
    int fmax = 0;
    for (int b = 0; b < e->B; ++b) {
      const long long* q = &ph[(size_t)b * 32];
      tot[b] = (double)(q[9] - q[0]);
      for (int k = 1; k < 10; ++k) pmax[k] = std::max(pmax[k], (double)(q[k] - q[k - 1]));
      fmax = std::max(fmax, (int)q[12]);
    }
    std::sort(tot.begin(), tot.end());
    std::fprintf(stderr, " | total mean=%.0f p50=%.0f p90=%.0f max=%.0f | phase max:",
                 std::accumulate(tot.begin(), tot.end(), 0.0) / e->B, tot[e->B / 2],
                 tot[(size_t)(e->B * 9 / 10)], tot.back());
    for (int k = 1; k < 10; ++k) std::fprintf(stderr, " p%d=%.0f", k, pmax[k]);
    std::fprintf(stderr, " flagged max=%d\n", fmax);
  }
  return MV_OK;
}

int mv_set_crossover(mv_engine* e, int32_t kind, double eta, double prob) {
  if (!e || kind < 0 || kind > 1 || !(eta >= 0.0) || !(prob >= 0.0 && prob <= 1.0))
    return fail(MV_ERR_ARG, "crossover: kind 0 (two-point) or 1 (SBX), eta >= 0, 0 <= prob <= 1");
  e->cx_kind = kind;
  e->sbx_eta = eta;
  e->cx_prob = prob;
  return MV_OK;
}

int mv_set_state_streams(mv_engine* e, int32_t enabled, int64_t first_state) {
  if (!e || enabled < 0 || enabled > 1 || first_state < 0 || first_state > 0x7FFFFFFF)
    return fail(MV_ERR_ARG, "state streams: enabled 0 or 1, 0 <= first_state < 2^31");
  e->state_keys = enabled;
  e->key0 = (uint32_t)first_state;
  return MV_OK;
}

int mv_set_mlp_precision(mv_engine* e, int32_t bf16) {
  if (!e || bf16 < 0 || bf16 > 1) return fail(MV_ERR_ARG, "mlp precision: 0 (fp32) or 1 (bf16)");
  if (bf16 && !e->has_model) return fail(MV_ERR_STATE, "no device classifier to run in bf16");
  e->mlp_bf16 = bf16;
  return MV_OK;
}

int mv_set_attack_mode(mv_engine* e, int32_t mode) {
  if (!e || mode < 0 || mode > 1)
    return fail(MV_ERR_ARG, "attack mode must be 0 (auto) or 1 (chain); the whole-attack "
                            "kernel (2) was retired: it measured slower than the chain");
  e->attack_mode = mode;
  return MV_OK;
}

int mv_get_attack_time(mv_engine* e, double* ms, int32_t* whole) {
  if (!e) return fail(MV_ERR_ARG, "null engine");
  if (whole) *whole = 0;
  if (ms) *ms = 0.0;
  return MV_OK;
}

int mv_det_pow(int64_t n, const double* x, const double* y, double* out) {
  if (n < 0 || (n > 0 && (!x || !y || !out))) return fail(MV_ERR_ARG, "bad mv_det_pow arguments");
  for (int64_t i = 0; i < n; ++i) out[i] = det_pow(x[i], y[i]);
  return MV_OK;
}

int mv_get_phase_times(mv_engine* e, double* ms, int32_t* n_generations) {
  if (!e || !ms) return fail(MV_ERR_ARG, "null argument");
  double t[4] = {0, 0, 0, 0};
  for (int i = 0; i < e->n_var_rec; ++i) {
    float a = 0.f, b = 0.f, c = 0.f;
    const hipEvent_t* kx = &e->ev_kx[6 * (size_t)i];
    HIPCHK(hipEventSynchronize(kx[5]));
    HIPCHK(hipEventElapsedTime(&a, kx[0], kx[1]));
    HIPCHK(hipEventElapsedTime(&b, kx[2], kx[3]));
    HIPCHK(hipEventElapsedTime(&c, kx[4], kx[5]));
    t[0] += a;
    t[1] += b;
    t[2] += c;
  }
  for (int i = 0; i < e->n_surv_rec; ++i) {
    float s = 0.f;
    HIPCHK(hipEventSynchronize(e->ev_surv[2 * i + 1]));
    HIPCHK(hipEventElapsedTime(&s, e->ev_surv[2 * i], e->ev_surv[2 * i + 1]));
    t[3] += s;
  }
  for (int k = 0; k < 4; ++k) ms[k] = t[k];
  if (n_generations) *n_generations = e->n_var_rec < e->n_surv_rec ? e->n_var_rec : e->n_surv_rec;
  return MV_OK;
}

struct mv_mlp {
  int device = 0;
  MlpArgs a{};
  std::vector<void*> allocs;
  ~mv_mlp() {
    (void)hipSetDevice(device);
    for (void* x : allocs) (void)hipFree(x);
  }
};

int mv_mlp_create(int32_t device, const mv_model_desc* md, mv_mlp** out) {
  if (!md || !out) return fail(MV_ERR_ARG, "null argument");
  *out = nullptr;
  if (md->n_layers < 2 || md->n_layers > MAX_LAYERS) return fail(MV_ERR_ARG, "2..6 layers");
  for (int l = 1; l < md->n_layers; ++l)
    if (md->dims[l] % 16 != 0 || md->dims[l] > 512)
      return fail(MV_ERR_ARG, "hidden widths must be multiples of 16 and <= 512");
  if (md->dims[md->n_layers] < 1 || md->dims[md->n_layers] > 8)
    return fail(MV_ERR_ARG, "output width must be 1..8");
  HIPCHK(hipSetDevice(device));
  mv_mlp* m = new mv_mlp();
  m->device = device;
  MlpArgs& a = m->a;
  a.n_layers = md->n_layers;
  for (int l = 0; l <= md->n_layers; ++l) a.dims[l] = md->dims[l];
  a.D4 = (md->dims[0] + 3) & ~3;
  int hmax = 16;
  for (int l = 1; l < a.n_layers; ++l) hmax = a.dims[l] > hmax ? a.dims[l] : hmax;
  if (predict_lds_bytes(a.D4, hmax, a.dims[a.n_layers - 1], a.dims[a.n_layers], 16) > 160 * 1024) {
    delete m;
    return fail(MV_ERR_ARG, "model input too wide for the LDS tile");
  }
  hipError_t err = hipSuccess;
  auto K = [&](auto** dst, const auto* host, size_t n) {
    if (err != hipSuccess) return;
    err = upload(dst, host, n);
    if (err == hipSuccess) m->allocs.push_back((void*)*dst);
  };
  std::vector<float> w0((size_t)a.D4 * a.dims[1], 0.f);
  std::memcpy(w0.data(), md->W[0], (size_t)a.dims[0] * a.dims[1] * sizeof(float));
  K((float**)&a.W[0], w0.data(), w0.size());
  K((float**)&a.bias[0], md->b[0], a.dims[1]);
  for (int l = 1; l < a.n_layers; ++l) {
    K((float**)&a.W[l], md->W[l], (size_t)a.dims[l] * a.dims[l + 1]);
    K((float**)&a.bias[l], md->b[l], a.dims[l + 1]);
  }
  if (err != hipSuccess) {
    delete m;
    return fail(MV_ERR_HIP, std::string("upload: ") + hipGetErrorString(err));
  }
  *out = m;
  return MV_OK;
}

void mv_mlp_destroy(mv_mlp* m) { delete m; }

int mv_mlp_predict(mv_mlp* m, int32_t n, const double* x, double* proba, void* stream) {
  if (!m || n < 0 || (n > 0 && (!x || !proba))) return fail(MV_ERR_ARG, "bad mv_mlp_predict");
  if (!on_device(x, m->device) || !on_device(proba, m->device))
    return fail(MV_ERR_ARG, "mv_mlp_predict: a buffer lives on another device than the classifier");
  HIPCHK(hipSetDevice(m->device));
  MlpArgs a = m->a;
  a.n = n;
  a.x = x;
  a.proba = proba;
  HIPCHK(launch_predict(a, (hipStream_t)stream));
  return MV_OK;
}

struct mv_objcalc {
  int device = 0;
  int D = 0, n_ohe = 0, norm = 2;
  int* ohe_off = nullptr;
  int* ohe_feat = nullptr;
  double *mm_s = nullptr, *mm_m = nullptr, *ml_s = nullptr, *ml_m = nullptr;
  double *xml = nullptr, *G = nullptr, *proba = nullptr;
  size_t cap_xml = 0, cap_G = 0, cap_p = 0;
  std::vector<void*> allocs;
  ~mv_objcalc() {
    (void)hipSetDevice(device);
    for (void* x : allocs) (void)hipFree(x);
    (void)hipFree(xml);
    (void)hipFree(G);
    (void)hipFree(proba);
  }
};

int mv_objcalc_create(int32_t device, const mv_objcalc_desc* d, mv_objcalc** out) {
  if (!d || !out || d->D <= 0 || d->n_ohe < 0 || !d->mm_scale || !d->mm_min ||
      (d->n_ohe > 0 && (!d->ohe_offsets || !d->ohe_feats)) ||
      ((d->ml_scale == nullptr) != (d->ml_min == nullptr)) || (d->norm != 2 && d->norm != 0))
    return fail(MV_ERR_ARG, "bad mv_objcalc_desc");
  *out = nullptr;
  for (int g = 0; g < d->n_ohe; ++g)
    if (d->ohe_offsets[g + 1] < d->ohe_offsets[g]) return fail(MV_ERR_ARG, "ohe offsets");
  const int nf = d->n_ohe > 0 ? d->ohe_offsets[d->n_ohe] : 0;
  for (int k = 0; k < nf; ++k)
    if (d->ohe_feats[k] < 0 || d->ohe_feats[k] >= d->D) return fail(MV_ERR_ARG, "ohe feature");
  HIPCHK(hipSetDevice(device));
  mv_objcalc* o = new mv_objcalc();
  o->device = device;
  o->D = d->D;
  o->n_ohe = d->n_ohe;
  o->norm = d->norm;
  std::vector<int> off(d->n_ohe + 1, 0), feat(nf > 0 ? nf : 1, 0);
  for (int g = 0; g <= d->n_ohe && d->n_ohe > 0; ++g) off[g] = d->ohe_offsets[g];
  for (int k = 0; k < nf; ++k) feat[k] = d->ohe_feats[k];
  hipError_t err = hipSuccess;
  auto K = [&](auto** dst, const auto* host, size_t n) {
    if (err != hipSuccess) return;
    err = upload(dst, host, n);
    if (err == hipSuccess) o->allocs.push_back((void*)*dst);
  };
  K(&o->ohe_off, off.data(), off.size());
  K(&o->ohe_feat, feat.data(), feat.size());
  K(&o->mm_s, d->mm_scale, (size_t)d->D);
  K(&o->mm_m, d->mm_min, (size_t)d->D);
  if (d->ml_scale) {
    K(&o->ml_s, d->ml_scale, (size_t)d->D);
    K(&o->ml_m, d->ml_min, (size_t)d->D);
  }
  if (err != hipSuccess) {
    delete o;
    return fail(MV_ERR_HIP, std::string("upload: ") + hipGetErrorString(err));
  }
  *out = o;
  return MV_OK;
}

void mv_objcalc_destroy(mv_objcalc* o) { delete o; }

static hipError_t grow(double** p, size_t* cap, size_t n) {
  if (n <= *cap) return hipSuccess;
  hipError_t e = hipDeviceSynchronize();  // earlier launches may still read the old buffer
  if (e != hipSuccess) return e;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  e = hipMalloc((void**)p, n * sizeof(double));
  if (e == hipSuccess) *cap = n;
  return e;
}

int mv_objcalc_run(mv_objcalc* o, mv_engine* e, mv_mlp* m, int32_t B, int32_t n,
                   const double* x_init, const double* x, int32_t minimize_class, double* obj,
                   int32_t* range_bad, void* stream_) {
  if (!o || !e || !m || B < 0 || n < 0) return fail(MV_ERR_ARG, "bad mv_objcalc_run arguments");
  if (e->p.D != o->D || m->a.dims[0] != o->D)
    return fail(MV_ERR_ARG, "constraints / classifier / scaler feature counts differ");
  const int n_out = m->a.dims[m->a.n_layers];
  if (minimize_class < 0 || minimize_class >= (n_out == 1 ? 2 : n_out))
    return fail(MV_ERR_ARG, "minimize_class outside the classifier output");
  const long total = (long)B * n;
  if (total == 0) return MV_OK;
  if (!x_init || !x || !obj || !range_bad) return fail(MV_ERR_ARG, "null buffer");
  if (e->device != o->device || m->device != o->device)
    return fail(MV_ERR_ARG, "objects live on different devices");
  if (!on_device(x_init, o->device) || !on_device(x, o->device) || !on_device(obj, o->device) ||
      !on_device(range_bad, o->device))
    return fail(MV_ERR_ARG, "mv_objcalc_run: a buffer lives on another device than the objects");
  hipStream_t stream = (hipStream_t)stream_;
  HIPCHK(hipSetDevice(o->device));
  HIPCHK(grow(&o->G, &o->cap_G, (size_t)total * (e->p.C > 0 ? e->p.C : 1)));
  HIPCHK(grow(&o->proba, &o->cap_p, (size_t)total * n_out));
  const double* xml = x;
  if (o->ml_s) {
    HIPCHK(grow(&o->xml, &o->cap_xml, (size_t)total * o->D));
    HIPCHK(launch_obj_mlscale(total * o->D, o->D, x, o->ml_s, o->ml_m, o->xml, stream));
    xml = o->xml;
  }
  if (e->p.C > 0) {
    int slot = 0;
    HIPCHK(stage_rows(base_rows(e), stream, &slot));
    HIPCHK(launch_constraints(e->p, slot, (int)total, x, o->G, stream));
    HIPCHK(release_rows(slot, stream));
  }
  MlpArgs ma = m->a;
  ma.n = (int)total;
  ma.x = xml;
  ma.proba = o->proba;
  HIPCHK(launch_predict(ma, stream));
  ObjArgs a{};
  a.total = total;
  a.n = n;
  a.D = o->D;
  a.C = e->p.C;
  a.n_ohe = o->n_ohe;
  a.n_out = n_out;
  a.cls = minimize_class;
  a.norm = o->norm;
  a.x = x;
  a.x_init = x_init;
  a.mm_scale = o->mm_s;
  a.mm_min = o->mm_m;
  a.ohe_off = o->ohe_off;
  a.ohe_feat = o->ohe_feat;
  a.G = o->G;
  a.proba = o->proba;
  a.obj = obj;
  a.range_bad = range_bad;
  HIPCHK(launch_objectives(a, stream));
  return MV_OK;
}

int mv_objcalc_score(mv_objcalc* o, int32_t B, int32_t n, const double* x_init, const double* x,
                     const double* G, int32_t C, const double* proba, int32_t n_out,
                     int32_t minimize_class, double* obj, int32_t* range_bad, void* stream_) {
  if (!o || B < 0 || n < 0 || C < 0 || n_out < 1)
    return fail(MV_ERR_ARG, "bad mv_objcalc_score arguments");
  if (minimize_class < 0 || minimize_class >= (n_out == 1 ? 2 : n_out))
    return fail(MV_ERR_ARG, "minimize_class outside the classifier output");
  const long total = (long)B * n;
  if (total == 0) return MV_OK;
  if (!x_init || !x || !obj || !range_bad || !proba || (C > 0 && !G))
    return fail(MV_ERR_ARG, "null buffer");
  if (!on_device(x_init, o->device) || !on_device(x, o->device) || !on_device(G, o->device) ||
      !on_device(proba, o->device) || !on_device(obj, o->device) || !on_device(range_bad, o->device))
    return fail(MV_ERR_ARG, "mv_objcalc_score: a buffer lives on another device than the calculator");
  HIPCHK(hipSetDevice(o->device));
  ObjArgs a{};
  a.total = total;
  a.n = n;
  a.D = o->D;
  a.C = C;
  a.n_ohe = o->n_ohe;
  a.n_out = n_out;
  a.cls = minimize_class;
  a.norm = o->norm;
  a.x = x;
  a.x_init = x_init;
  a.mm_scale = o->mm_s;
  a.mm_min = o->mm_m;
  a.ohe_off = o->ohe_off;
  a.ohe_feat = o->ohe_feat;
  a.G = G;
  a.proba = proba;
  a.obj = obj;
  a.range_bad = range_bad;
  HIPCHK(launch_objectives(a, (hipStream_t)stream_));
  return MV_OK;
}

int mv_debug_checks(int32_t* record, int32_t* compiled) {
  if (!record) return fail(MV_ERR_ARG, "null record");
  if (compiled) *compiled = MV_CHECKS_ON;
  HIPCHK(hipDeviceSynchronize());
  int ev[8], sv[8];
  HIPCHK(take_checks_eval(ev));
  HIPCHK(take_checks_survive(sv));
  const int* r = ev[0] ? ev : sv;
  for (int k = 0; k < 8; ++k) record[k] = r[k];
  record[5] = ev[5] + sv[5];
  return MV_OK;
}

int mv_debug_survival_dump(double* out) {
  if (!out) return fail(MV_ERR_ARG, "null dump buffer");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(take_survival_dump(out));
  return MV_OK;
}

int mv_attack_population(mv_engine* e, double* genes, double* F, void* stream) {
  if (!e || !e->attack_ready) return fail(MV_ERR_STATE, "no attack has run");
  if (!on_device(genes, e->device) || !on_device(F, e->device))
    return fail(MV_ERR_ARG, "mv_attack_population: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  // the pool's rows in the attack's layout -> genes of every one of the Vr genes
  const DProblem& ap = e->ap();
  const int* cmap = ap.compact ? (const int*)(ap.vblob + vary_offsets(ap).cmap) : nullptr;
  HIPCHK(launch_gather_pop(e->B, e->P, ap.V, ap.Vr, e->S, cmap, e->s.gl, e->pop_slot, e->pool,
                           e->poolF, genes, F, (hipStream_t)stream));
  if (MV_CHECKS_ON) {  // checks build: a failed device index check fails the attack loudly
    int32_t r[8];
    if (mv_debug_checks(r, nullptr) != MV_OK) return MV_ERR_HIP;
    if (r[0])
      return fail(MV_ERR_STATE, "device index check " + std::to_string(r[0]) + " failed (block " +
                                    std::to_string(r[1]) + ", thread " + std::to_string(r[2]) +
                                    ", value " + std::to_string(r[3]) + ", bound " +
                                    std::to_string(r[4]) + ", " + std::to_string(r[5]) +
                                    " failures)");
  }
  return MV_OK;
}

int mv_attack_front(mv_engine* e, uint8_t* front, int32_t* offsets, double* X, double* Fx,
                    void* stream) {
  if (!e || !e->attack_ready) return fail(MV_ERR_STATE, "no attack has run");
  if (!on_device(front, e->device) || !on_device(offsets, e->device) ||
      !on_device(X, e->device) || !on_device(Fx, e->device))
    return fail(MV_ERR_ARG, "mv_attack_front: a buffer lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  if (!front || !offsets) {  // scratch for the mask / offsets the caller does not want
    if (!e->front_scr) {
      hipError_t err = dalloc(&e->front_scr, (size_t)e->B * e->P);
      if (err == hipSuccess) e->attack_allocs.push_back(e->front_scr);
      if (err == hipSuccess) err = dalloc(&e->off_scr, (size_t)e->B + 1);
      if (err == hipSuccess) e->attack_allocs.push_back(e->off_scr);
      if (err != hipSuccess) return fail(MV_ERR_HIP, std::string("alloc: ") + hipGetErrorString(err));
    }
    if (!front) front = e->front_scr;
    if (!offsets) offsets = e->off_scr;
  }
  const DProblem& ap = e->ap();
  const int* cmap = ap.compact ? (const int*)(ap.vblob + vary_offsets(ap).cmap) : nullptr;
  HIPCHK(launch_front(e->B, e->P, ap.V, ap.Vr, e->S, cmap, e->s.gl, e->pop_slot, e->pool,
                      e->poolF, front, offsets, X, Fx, (hipStream_t)stream));
  return MV_OK;
}

int mv_gene_layout(mv_engine* e, int32_t B, const double* x_init, const double* xl,
                   const double* xu, int32_t* stored, int32_t* n_stored) {
  if (!e || B < 0 || (B > 0 && (!x_init || !xl || !xu)) || !stored || !n_stored)
    return fail(MV_ERR_ARG, "bad mv_gene_layout arguments");
  const std::vector<int> keep = B > 0 ? stored_genes(e, B, x_init, xl, xu) : std::vector<int>{};
  for (int g = 0; g < e->hp.V; ++g) stored[g] = keep.empty() ? 1 : 0;
  for (int g : keep) stored[g] = 1;
  *n_stored = keep.empty() ? e->hp.V : (int32_t)keep.size();
  return MV_OK;
}

int mv_set_gene_layout(mv_engine* e, const int32_t* stored, int32_t V) {
  if (!e) return fail(MV_ERR_ARG, "null engine");
  if (!stored) {
    e->layout_req.clear();
    return MV_OK;
  }
  if (V != e->hp.V) return fail(MV_ERR_ARG, "mv_set_gene_layout: V differs from the problem's");
  std::vector<int> keep;
  for (int g = 0; g < V; ++g)
    if (stored[g]) keep.push_back(g);
  if (keep.empty()) return fail(MV_ERR_ARG, "mv_set_gene_layout: no stored gene");
  e->layout_req = keep;
  return MV_OK;
}

int mv_get_stored_genes(mv_engine* e, int32_t* stored, int32_t* n_stored) {
  if (!e || !n_stored) return fail(MV_ERR_ARG, "null argument");
  const DProblem& ap = e->ap();
  *n_stored = ap.V;
  if (stored)
    for (int g = 0; g < ap.Vr; ++g) {
      const auto it = std::lower_bound(e->stored.begin(), e->stored.end(), g);
      stored[g] = !ap.compact || (it != e->stored.end() && *it == g);
    }
  return MV_OK;
}

int mv_attack_history(mv_engine* e, double* hist, void* stream) {
  if (!e || !e->attack_ready || !e->hist_mode) return fail(MV_ERR_STATE, "no history recorded");
  if (!hist) return fail(MV_ERR_ARG, "null hist");
  if (!on_device(hist, e->device))
    return fail(MV_ERR_ARG, "mv_attack_history: hist lives on another device than the engine");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipMemcpyAsync(hist, e->hist, (size_t)e->B * e->hist_rows * e->hist_w * sizeof(double),
                        hipMemcpyDefault, (hipStream_t)stream));
  return MV_OK;
}

}  // extern "C"
