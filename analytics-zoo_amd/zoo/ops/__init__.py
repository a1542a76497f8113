"""zoo.ops — functional ops backed by the hand-written gfx950 HIP kernels.

GPU tensors run on the native kernels in ``zoo._C`` (fail loudly if missing);
CPU tensors run on PyTorch reference implementations (used by the CPU test
suite and as numerics oracles).
"""
from zoo.ops._native import native, available, set_deterministic, deterministic
from zoo.ops.conv import conv2d_nhwc, linear, pack_weight, unpack_weight, ceil8, conv_out_size
from zoo.ops.bn import conv_bn_act, batch_norm_nhwc, GradHandoff, BNProducer
from zoo.ops.pool import max_pool2d_nhwc, global_avg_pool_nhwc
from zoo.ops.loss import prob_nll, softmax_cross_entropy
from zoo.ops.nn import layer_norm, embedding, dropout_add, depthwise_conv2d_nhwc, lrn_channels_last
from zoo.ops.attention import attention
