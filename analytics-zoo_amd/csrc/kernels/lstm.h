// LSTM gate activations shared by the ConvLSTM kernels (keras_ops.hip, convlstm.hip).
#pragma once
#include "common.h"

namespace zoo {

// activation codes (zoo/ops/layers.py): 0 linear, 1 tanh, 2 sigmoid, 3 hard_sigmoid, 4 relu
ZOO_DEV float lstm_act(float x, int a) {
  switch (a) {
    case 1: return tanhf(x);
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: { const float v = 0.2f * x + 0.5f; return v < 0.f ? 0.f : (v > 1.f ? 1.f : v); }
    case 4: return x > 0.f ? x : 0.f;
    default: return x;
  }
}
// derivative from the activation's OUTPUT
ZOO_DEV float lstm_dact(float y, int a) {
  switch (a) {
    case 1: return 1.f - y * y;
    case 2: return y * (1.f - y);
    case 3: return (y > 0.f && y < 1.f) ? 0.2f : 0.f;
    case 4: return y > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

}  // namespace zoo
