// ntt_conv12.hip -- forward column passes with the 1- and 2-source conversion prologue (PRO_CONV)
// (kernel templates: ntt_core.hpp; one translation unit per entry-point family so
// the ~360 pass kernels compile in parallel)
#include "ntt_core.hpp"

int ntt_conv_col12(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  if (a.c_ns == 1) return col_pass<PRO_CONV>(c, a, false, n_jobs);
  return col_pass<PRO_CONV + 1>(c, a, false, n_jobs);
}
