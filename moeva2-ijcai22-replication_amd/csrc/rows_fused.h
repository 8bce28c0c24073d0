// Fused row kernel body (variation + decode + f2 + constraint program) shared by k_rows
// (eval.hip, one workgroup per chunk of a state's rows) and the whole-attack kernel
// (attack_impl.h, one workgroup per state).
#pragma once
#include "engine.h"
#include "kernels.h"
#include "philox.h"
#include "rowops.h"
#include "wave.h"

namespace mv {

// ---------------------------------------------------------------------------------------
// Fused row phase: k_gen + k_cons for rows [r0, r1) of state b on the workgroup's W waves.
// Wave w takes rows c0 + w + W k of each chunk of 64 W rows (lane k of the wave holds row
// k's parents, crossover draws and cached mutations, exactly as k_gen).  Every table the
// row loop reads is staged in LDS first: a global load inside the loop would make the wave
// wait (vmcnt is in order) for the next row's prefetched parent genes too.
template <bool IDENT, int NT, bool FULL, int T>
__device__ __forceinline__ void rows_state(const RowsArgs& a, const int b, const int gen,
                                           const int hist_row0, const int r0, const int r1,
                                           unsigned char* smem) {
  constexpr int W = T / 64;
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // uniform by construction; readfirstlane lets the non-inlined phase keep them in SGPRs
  const int V = __builtin_amdgcn_readfirstlane(p.V);
  const int Dm = __builtin_amdgcn_readfirstlane(p.Dm);
  const int Dm4 = __builtin_amdgcn_readfirstlane(p.Dm4);
  const VaryOff o = vary_offsets(p);
  const FusedLds L = fused_lds(o, W);
  const unsigned char* sblob = a.s.sblob + (size_t)b * o.sb;
  glds_copy<T>(smem + L.a_at, p.vblob, o.a_end, wave, lane);
  glds_copy<T>(smem + L.b_at, p.vblob + o.b_at, o.b_end - o.b_at, wave, lane);
  glds_copy<T>(smem + L.c_at, p.vblob + o.c_at, o.vb - o.c_at, wave, lane);
  glds_copy<T>(smem + L.e_at, sblob + o.e_at, o.sb - o.e_at, wave, lane);
  int ginf[NT];
  {
    const int* gi = (const int*)(p.vblob + o.ginfo);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int g = lane + 64 * t;
      const int w = gi[g < V ? g : V - 1];  // unconditional load (see k_cons load_row)
      ginf[t] = g < V ? w : 0;
    }
  }
  // the wave's ML-space row buffer: immutable features from x_init (written once)
  double* xrow = (double*)(smem + L.rows_at + wave * o.rb);
  {
    const double* xi = (const double*)(sblob + o.xi);
    for (int f = lane; f < p.D; f += 64) xrow[f] = xi[f];
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  // constraint program (LDS) and this lane's ops packed in registers
  OpTab tab;
  tab.code = (const int*)(smem + L.a_at + o.opc);
  tab.arg = (const int4*)(smem + L.a_at + o.opa);
  tab.k = (const double2*)(smem + L.a_at + o.opk);
  tab.col = (const int*)(smem + L.a_at + o.ocol);
  tab.pool = (const int*)(smem + L.a_at + o.pool);
  tab.C = p.C;
  tab.n_lane = p.C - p.n_sumdiff;
  tab.tol = p.tol;
  unsigned opw[OPS_REG];
  const int kops = min(OPS_REG, (tab.n_lane + 63) >> 6);
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    const int c = lane + 64 * k;
    opw[k] = (k < kops && c < tab.n_lane) ? pack_op(tab, c) : 0u;
  }
  const int* s_ooff = (const int*)(smem + L.b_at + (o.ooff - o.b_at));
  const int* s_ofeat = (const int*)(smem + L.b_at + (o.ofeat - o.b_at));
  const int* s_ginfo = (const int*)(smem + L.b_at + (o.ginfo - o.b_at));
  const uint32_t* s_geo = (const uint32_t*)(smem + L.b_at + (o.geo - o.b_at));
  const int* s_mutf = (const int*)(smem + L.b_at + (o.mutf - o.b_at));
  const double* s_mlS = (const double*)(smem + L.c_at + (o.mlS - o.c_at));
  const double* s_mlM = (const double*)(smem + L.c_at + (o.mlM - o.c_at));
  const double* s_es = (const double*)(smem + L.e_at + (o.es - o.e_at));
  const double* s_em = (const double*)(smem + L.e_at + (o.em - o.e_at));
  const double* s_x0 = (const double*)(smem + L.e_at + (o.x0 - o.e_at));
  const double* gin = a.genes_in + (size_t)b * a.in_rows * V;
  const bool l2 = p.norm == 2;
  const Rng rng(a.seed, a.stream_key);
  const double* sgl = a.s.gl + (size_t)b * V;  // genetic bounds (SBX rows read all of them)
  const double* sgu = a.s.gu + (size_t)b * V;
  const bool sbx = a.mode == 1 && a.cx_kind == 1;
  for (int c0 = r0; c0 < r1; c0 += 64 * W) {
    const int span = min(r1, c0 + 64 * W) - c0 - wave;
    const int nrw = span > 0 ? (span + W - 1) / W : 0;
    // lane k: row k's packed parents (own | oth << 16), crossover draws, destination and
    // mutations (count | overflow << 3 | (last position + 1) << 4)
    int par_v = 0, cx0_v = 0, cx1_v = 0, orow_v = 0, mut_v = 0;
    int mpos[MUT_CAP];
    double mval[MUT_CAP];
#pragma unroll
    for (int q = 0; q < MUT_CAP; ++q) {
      mpos[q] = -1;
      mval[q] = 0.0;
    }
    const bool mine = lane < nrw;
    const int irow = c0 + wave + W * lane;
    if (mine) orow_v = a.out_map ? a.out_map[(size_t)b * a.n + irow] : irow;
    if (a.mode == 1) {
            if (mine) {
        const int nm = a.n / 2;
        const int m = irow % nm;
        const int side = irow / nm;
        const int2 pr = *(const int2*)(a.parents + ((size_t)b * nm + m) * 2);
        par_v = side ? (pr.y | (pr.x << 16)) : (pr.x | (pr.y << 16));
        cx0_v = pack_cx(cx_sub(rng, gen, m, 0, p.n_sub[0], a.cx_prob));
        cx1_v = pack_cx(cx_sub(rng, gen, m, 1, p.n_sub[1], a.cx_prob));
        if (sbx) {  // SBX: the subsets' mating-level draws only (no segment)
          cx0_v &= 1;
          cx1_v &= 1;
        }
      }
      const float lq = __log2f(1.0f - 1.0f / (float)V);
      bool going = mine && !sbx;
      int pos = -1, cnt = 0, ovf = 0;
      double mu[MUT_CAP];
#pragma unroll 1
      for (int j = 0; j <= MUT_CAP && __ballot(going); ++j) {
        bool have = false;
        double u = 0.0;
        if (going) {
          const u32x4 w = rng.draw((uint32_t)(irow * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
          pos += 1 + geo_gap(s_geo, V, w.x, lq);
          if (pos >= V) {
            going = false;
          } else if (j == MUT_CAP) {
            ovf = 1;
            going = false;
          } else {
            have = true;
            u = u53(w.y, w.z);
            cnt = j + 1;
          }
        }
#pragma unroll
        for (int q = 0; q < MUT_CAP; ++q)
          if (have && q == j) {
            mpos[q] = pos;
            mu[q] = u;
          }
      }
      const double* gl = a.s.gl + (size_t)b * V;
      const double* gu = a.s.gu + (size_t)b * V;
      double mlo[MUT_CAP], mhi[MUT_CAP];
#pragma unroll
      for (int q = 0; q < MUT_CAP; ++q) {
        const int mp = mpos[q] < 0 ? 0 : mpos[q];
        const bool sw = swapped_packed(s_ginfo[mp], cx0_v, cx1_v);
        mval[q] = gin[(size_t)(sw ? (par_v >> 16) : (par_v & 0xFFFF)) * V + mp];
        mlo[q] = gl[mp];
        mhi[q] = gu[mp];
      }
#pragma unroll 1
      for (int q = 0; q < MUT_CAP && __ballot(q < cnt); ++q) {
        int gp = 0;
        double xv = 0.0, u = 0.0, lo = 0.0, hi = 0.0;
#pragma unroll
        for (int r = 0; r < MUT_CAP; ++r)
          if (r == q) {
            gp = mpos[r];
            xv = mval[r];
            u = mu[r];
            lo = mlo[r];
            hi = mhi[r];
          }
        if (q < cnt) {
          xv = mutate_gene(xv, lo, hi, (s_ginfo[gp] & 3) == 0, u, a.eta);
#pragma unroll
          for (int r = 0; r < MUT_CAP; ++r)
            if (r == q) mval[r] = xv;
        }
      }
      int last = -1;
#pragma unroll
      for (int q = 0; q < MUT_CAP; ++q)
        if (q < cnt) last = mpos[q];
      mut_v = cnt | (ovf << 3) | ((last + 1) << 4);
    } else if (mine) {
      par_v = irow | (irow << 16);
    }
    auto load_row = [&](int k, double* x) {
      load_parent_row<NT>(gin, V, rdl(par_v, k), rdl(cx0_v, k), rdl(cx1_v, k), ginf, lane, x);
    };
    // child genes -> pool, fp32 ML row, f2, constraint program -> f3 (row k of this wave)
    auto finish_row = [&](int k, const double* x) {
      int Vo = V, Dmo = Dm, Dm4o = Dm4;
      asm volatile("" : "+s"(Vo), "+s"(Dmo), "+s"(Dm4o));
      const int i = c0 + wave + W * k;
      const int orow = rdl(orow_v, k);
      if (a.genes_out) {
        double* gout = a.genes_out + ((size_t)b * a.out_rows + orow) * V;
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (lane + 64 * t < Vo) gout[lane + 64 * t] = x[t];
      }
      // ML-space row in the wave's buffer (feature_encoder.py:91-124)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (lane + 64 * t < Vo) {
          if (IDENT)
            xrow[(ginf[t] >> 17) & 0x7FFF] = x[t];
          else
            scatter_gene_tab(s_ooff, s_ofeat, xrow, ginf[t], x[t]);
        }
      }
      wave_sync();
      float* xo = a.xml + ((size_t)b * (a.xml_rows ? a.xml_rows : a.n) + i) * Dm4;
      double acc = 0.0;
      if (IDENT) {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int j = lane + 64 * t;
          if (j < Dm4o) {
            float v = 0.f;
            if (j < Dmo) {
              const double xf = x[t];
              v = (float)(xf * s_mlS[j] + s_mlM[j]);
              const double d = (xf * s_es[j] + s_em[j]) - s_x0[j];
              acc = l2 ? acc + d * d : nanmax(acc, fabs(d));
            }
            xo[j] = v;
          }
        }
      } else {
        for (int j = lane; j < Dm4; j += 64) {
          float v = 0.f;
          if (j < Dm) {
            const double xf = xrow[s_mutf[j]];
            v = (float)(xf * s_mlS[j] + s_mlM[j]);
            const double d = (xf * s_es[j] + s_em[j]) - s_x0[j];
            acc = l2 ? acc + d * d : nanmax(acc, fabs(d));
          }
          xo[j] = v;
        }
      }
      acc = l2 ? wave_sum(acc) : wave_max(acc);
      double* grow = a.G ? a.G + ((size_t)b * a.n + i) * p.C : nullptr;
      double* hrow =
          a.hist ? a.hist + ((size_t)b * a.hist_rows + hist_row0 + i) * a.hist_w : nullptr;
      const double f3 = constraints_regs<FULL>(tab, opw, kops, xrow, lane, grow,
                                               (hrow && a.hist_w > 3) ? hrow + 3 : nullptr);
      if (lane == 0) {
        double f2 = l2 ? sqrt(acc) : acc;
        if (p.scale_obj) f2 = f2 * p.f2_scale + 0.0;
        if (a.F) {
          a.F[((size_t)b * a.out_rows + orow) * 3 + 1] = f2;
          a.F[((size_t)b * a.out_rows + orow) * 3 + 2] = f3;
        }
        if (hrow) {
          hrow[1] = f2;
          hrow[2] = f3;
        }
      }
      wave_sync();  // the next row overwrites xrow
    };
    double xn[NT];
    if (nrw > 0) load_row(0, xn);
    for (int k = 0; k < nrw; ++k) {
      double x[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) x[t] = xn[t];
      if (k + 1 < nrw) load_row(k + 1, xn);
      if (sbx) {  // SBX children, then every mutation of the row
        const int i = c0 + wave + W * k;
        const int nm = a.n / 2;
        const int pr = rdl(par_v, k);
        sbx_row<NT>(x, ginf, gin + (size_t)(pr >> 16) * V, sgl, sgu, V, i % nm, i / nm,
                    rdl(cx0_v, k) & 1, rdl(cx1_v, k) & 1, rng, gen, a.sbx_eta, lane);
        mutate_row_full<NT>(x, s_geo, s_ginfo, sgl, sgu, V, i, rng, gen, a.eta, lane);
      } else if (a.mode == 1) {
        apply_row_mutations<NT>(x, rdl(mut_v, k) & 7, mpos, mval, k, lane);
      }
      finish_row(k, x);
    }
    // rare: rows with more than MUT_CAP mutations are redone with every mutation
    if (a.mode == 1 && __ballot(mut_v & 8)) {
      const RowsArgs* ap = &a;
      const uint64_t seed2 = *(volatile const uint64_t*)&ap->seed;
      const Rng rng2(seed2, a.stream_key);
      const double* gl = a.s.gl + (size_t)b * V;
      const double* gu = a.s.gu + (size_t)b * V;
      const float lq = __log2f(1.0f - 1.0f / (float)V);
      for (int k = 0; k < nrw; ++k) {
        if (!(rdl(mut_v, k) & 8)) continue;
        const int i = c0 + wave + W * k;
        double x[NT];
        load_row(k, x);
        int pos = -1;
        for (int j = 0;; ++j) {
          const u32x4 w = rng2.draw((uint32_t)(i * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
          pos += 1 + geo_gap(s_geo, V, w.x, lq);
          if (pos >= V) break;
          double xv = 0.0;
#pragma unroll
          for (int t = 0; t < NT; ++t)
            if (pos == lane + 64 * t) xv = x[t];
          if ((pos & 63) == lane) {
            xv = mutate_gene(xv, gl[pos], gu[pos], (s_ginfo[pos] & 3) == 0, u53(w.y, w.z), a.eta);
#pragma unroll
            for (int t = 0; t < NT; ++t)
              if (pos == lane + 64 * t) x[t] = xv;
          }
        }
        finish_row(k, x);
      }
    }
  }
}

}  // namespace mv
