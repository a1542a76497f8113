// Host / device argument block of the fused NeuralCF kernels (ncf.hip).
#pragma once
#include <stdint.h>

namespace zoo {

struct NcfArgs {
  const int64_t* ids;  // [B, 2] (user, item)
  int B, id_off;
  const void *tu, *ti, *tmu, *tmi;  // embedding tables [V, e] (T)
  int Vu, Vi, eu, ei, em;           // em == 0: no matrix-factorisation branch
  const float *w1, *b1, *w2, *b2, *w3, *b3, *wo, *bo;
  int h1, h2, h3, nc;
  float* probs;         // forward output [B, nc]
  const float* dprobs;  // backward input [B, nc]
  float *gtu, *gti, *gtmu, *gtmi;
  float* partial;       // [gridDim.x, nwg] packed weight-gradient partials
  int nwg;
};

}  // namespace zoo
