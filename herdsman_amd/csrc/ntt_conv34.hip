// ntt_conv34.hip -- forward column passes with the 3- and 4-source conversion prologue (PRO_CONV), and the dispatch over ns
// (kernel templates: ntt_core.hpp; one translation unit per entry-point family so
// the ~360 pass kernels compile in parallel)
#include "ntt_core.hpp"

// the forward column pass with the conversion prologue over a.c_ns sources
int ntt_conv_col(fhe_ctx *c, const NttArgs &a, u32 n_jobs) {
  switch (a.c_ns) {
    case 1:
    case 2: return ntt_conv_col12(c, a, n_jobs);
    case 3: return col_pass<PRO_CONV + 2>(c, a, false, n_jobs);
    case 4: return col_pass<PRO_CONV + 3>(c, a, false, n_jobs);
  }
  return fhe_fail(c, FHE_ERR_UNSUPPORTED, "conversion prologue: 1..4 source limbs");
}
