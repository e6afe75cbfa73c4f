// gram_tab.hpp -- the table description of an additive kernel whose components are Cat / Bin gates times at
// most one RBF / periodic factor of an integer-coded covariate (gram.hip's table path, kl_hyper.hip's binned
// hyper-parameter gradient): per-workgroup LDS tables of the factors and their parameter derivatives as
// functions of (the pair's gate bits, the integer distance).
#pragma once
#include <climits>

#include "common.hpp"

namespace lvae {

constexpr float kLog2e = 1.4426950408889634f;
constexpr int kTabD = 64;

// sin(pi t) for t = |d| / p >= 0: reduced to pi r, r = t - rint(t) in [-1/2, 1/2] in fp64 (the
// period is exact), then the native sine (sin^2 has period pi, so the sign flip of the reduction
// cancels in every use; per_sin2 gives sin(2 pi t) = sin(2 pi r) for the period derivative)
__device__ inline float per_sin(double t) { return __sinf(float(M_PI) * float(t - rint(t))); }
__device__ inline float per_sin2(double t) { return __sinf(2.f * float(M_PI) * float(t - rint(t))); }

constexpr int kTabMaxG = 3, kTabMaxBits = 5;
constexpr int kTabR = kTabD + 1;  // table row stride (odd: the rows of different gate bits on other banks)
constexpr int kTabMaxFillLds = kTabMaxG * (1 << kTabMaxBits) * kTabR;  // floats
constexpr int kTabMaxBwdLds = 256 * kTabR;                             // floats (n_params 2^B <= 256)
struct GramTab {
  int ng, nbits, n_params;
  int gdim[kTabMaxG];                               // the group's continuous dim (-1: none at all)
  int bkind[kTabMaxBits], bdim[kTabMaxBits];        // gate b: LVAE_CAT / LVAE_BIN on dim
  int cgrp[LVAE_MAX_COMP], cmask[LVAE_MAX_COMP];    // component r: its group, the gate bits it needs
  int ckind[LVAE_MAX_COMP], cpi[LVAE_MAX_COMP];     // its continuous factor (kind -1: none), param index
  int csc[LVAE_MAX_COMP];                           // its scale's param index
  int n_comp;
  int porder[64];                                   // parameter slots ordered by group
  int pbeg[kTabMaxG + 1];                           // porder[pbeg[g] .. pbeg[g + 1]) belong to group g
  int pcomp[64], ptype[64];                         // slot p: its component, 0 scale / 1 RBF l / 2 PER l / 3 PER p
};

// host: the table description of spec, false if the spec does not fit it
static bool gram_tab_build(const lvae_kernel_spec* s, GramTab& t) {
  t = GramTab{};
  t.n_comp = s->n_comp;
  t.n_params = s->n_params;
  if (s->n_params > 64 || s->n_comp < 1) return false;
  for (int r = 0; r < s->n_comp; ++r) {
    int nc = 0, mask = 0;
    t.ckind[r] = -1;
    t.cpi[r] = 0;
    t.cgrp[r] = -1;
    t.csc[r] = s->scale_idx[r];
    for (int f = 0; f < s->n_fac[r]; ++f) {
      const int k = s->kind[r][f], d = s->dim[r][f];
      if (k == LVAE_CAT || k == LVAE_BIN) {
        int b = 0;
        while (b < t.nbits && !(t.bkind[b] == k && t.bdim[b] == d)) ++b;
        if (b == t.nbits) {
          if (t.nbits == kTabMaxBits) return false;
          t.bkind[b] = k;
          t.bdim[b] = d;
          ++t.nbits;
        }
        mask |= 1 << b;
      } else if (k == LVAE_RBF || k == LVAE_PER) {
        if (++nc > 1) return false;
        int g = 0;
        while (g < t.ng && t.gdim[g] != d) ++g;
        if (g == t.ng) {
          if (t.ng == kTabMaxG) return false;
          t.gdim[g] = d;
          ++t.ng;
        }
        t.cgrp[r] = g;
        t.ckind[r] = k;
        t.cpi[r] = s->param_idx[r][f];
      } else {
        return false;  // linear factors: not a function of the distance
      }
    }
    t.cmask[r] = mask;
  }
  if (t.ng == 0) {
    t.ng = 1;
    t.gdim[0] = -1;
  }
  for (int r = 0; r < s->n_comp; ++r)
    if (t.cgrp[r] < 0) t.cgrp[r] = 0;
  // parameter slots -> (component, type); ordered by group
  for (int p = 0; p < 64; ++p) t.pcomp[p] = -1;
  for (int r = 0; r < s->n_comp; ++r) {
    t.pcomp[t.csc[r]] = r;
    t.ptype[t.csc[r]] = 0;
    if (t.ckind[r] == LVAE_RBF) {
      t.pcomp[t.cpi[r]] = r;
      t.ptype[t.cpi[r]] = 1;
    } else if (t.ckind[r] == LVAE_PER) {
      t.pcomp[t.cpi[r]] = r;
      t.ptype[t.cpi[r]] = 2;
      t.pcomp[t.cpi[r] + 1] = r;
      t.ptype[t.cpi[r] + 1] = 3;
    }
  }
  int k = 0;
  for (int g = 0; g < t.ng; ++g) {
    t.pbeg[g] = k;
    for (int p = 0; p < s->n_params; ++p)
      if (t.pcomp[p] >= 0 && t.cgrp[t.pcomp[p]] == g) t.porder[k++] = p;
  }
  t.pbeg[t.ng] = k;
  if (t.ng * (1 << t.nbits) * kTabR > kTabMaxFillLds) return false;
  if (k * (1 << t.nbits) * kTabR > kTabMaxBwdLds) return false;
  return true;
}

// the continuous factor phi_r(m) of component r at integer distance m (1 without one), fp32 as the
// direct path (apply_factor); and the parts of its parameter derivatives the raw sums carry
__device__ inline float tab_phi(const GramTab& t, int r, const float* __restrict__ sp, int m) {
  const int k = t.ckind[r];
  if (k == LVAE_RBF) {
    const float ell = sp[t.cpi[r]], cf = -0.5f * kLog2e / (ell * ell), df = float(m);
    return __builtin_amdgcn_exp2f(cf * df * df);
  }
  if (k == LVAE_PER) {
    const float ell = sp[t.cpi[r]], cf = -2.f * kLog2e / (ell * ell);
    const float sn = per_sin((double)m / (double)sp[t.cpi[r] + 1]);
    return __builtin_amdgcn_exp2f(cf * sn * sn);
  }
  return 1.f;
}

// fill tables: tab[(g * 2^B + b) * kTabR + m] = sum over the components r of group g whose gates are in b
__device__ inline void tab_build_fill(const GramTab& t, const float* __restrict__ sp, float* __restrict__ tab) {
  const int nb = 1 << t.nbits, ne = t.ng * nb * kTabR;
  for (int e = threadIdx.x; e < ne; e += blockDim.x) {
    const int m = e % kTabR, b = (e / kTabR) % nb, g = e / (kTabR * nb);
    float v = 0.f;
    for (int r = 0; r < t.n_comp; ++r)
      if (t.cgrp[r] == g && (t.cmask[r] & ~b) == 0) v += sp[t.csc[r]] * tab_phi(t, r, sp, m);
    tab[e] = v;
  }
}

// adjoint tables: tab[(k * 2^B + b) * kTabR + m] for the k-th slot of porder: d k_r / d theta without
// the constants kl_gram_bwd_reduce applies (scale: phi; RBF l: s phi m^2; PER l: s phi sin^2 u; PER p:
// s phi m sin 2u), 0 when r's gates are not all in b
// entry e of the derivative tables (slot k = e / (kTabR 2^nbits), gate bits b, distance m)
__device__ inline float tab_bwd_entry(const GramTab& t, const float* __restrict__ sp, int e) {
  const int nb = 1 << t.nbits;
  {
    const int m = e % kTabR, b = (e / kTabR) % nb, k = e / (kTabR * nb);
    const int p = t.porder[k], r = t.pcomp[p], ty = t.ptype[p];
    float v = 0.f;
    if ((t.cmask[r] & ~b) == 0) {
      const float phi = tab_phi(t, r, sp, m), sc = sp[t.csc[r]];
      if (ty == 0) v = phi;
      else if (ty == 1) v = sc * phi * float(m) * float(m);
      else {
        const double u = (double)m / (double)sp[t.cpi[r] + 1];
        if (ty == 2) {
          const float sn = per_sin(u);
          v = sc * phi * sn * sn;
        } else {
          v = sc * phi * float(m) * per_sin2(u);
        }
      }
    }
    return v;
  }
}

__device__ inline void tab_build_bwd(const GramTab& t, const float* __restrict__ sp, float* __restrict__ tab) {
  const int ne = t.pbeg[t.ng] * (1 << t.nbits) * kTabR;
  for (int e = threadIdx.x; e < ne; e += blockDim.x) tab[e] = tab_bwd_entry(t, sp, e);
}

}  // namespace lvae
