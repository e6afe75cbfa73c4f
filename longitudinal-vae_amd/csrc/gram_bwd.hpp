// gram_bwd.hpp -- host descriptors of the batched Grams (gram.hip): up to 4 Grams in one forward launch
// (the Hensman forward), and up to 4 Grams contracted against their G in two launches (used by
// lvae_gram_bwd_f64 and the Hensman backward).
#pragma once
#include "common.hpp"

namespace lvae {

struct GramBwdJob {
  int spec;  // index into the specs[2] argument
  lvae_xview x1, x2;
  int nb, n1, n2, n_params;
  const double* params;
  const double* G;
  int64_t gsb, gsl, ldg;
  double* dparams;
  double* ddiag;
  int chunk0, nchunks;  // filled by gram_bwd_multi_f64
};

size_t gram_bwd_part_bytes(const GramBwdJob* jobs, int njobs, int L);

// forward: up to 4 fp64 Grams in one launch (gram_multi_f64; the Hensman forward's four), each as
// lvae_gram_f64's arguments (gx, gy, blk0 filled by gram_multi_f64)
struct GramFwdJob {
  int spec, nb, n1, n2, gx, gy, blk0;
  lvae_xview x1, x2;
  const double* params;
  const double* diag;
  double* out;
  int64_t osb, osl, ldo;
};
int gram_multi_f64(const lvae_kernel_spec* const* specs, const GramFwdJob* jobs, int njobs, int L, hipStream_t st);
int gram_bwd_multi_f64(const lvae_kernel_spec* const* specs, const GramBwdJob* jobs, int njobs, int L, double* part,
                       hipStream_t st);

}  // namespace lvae
