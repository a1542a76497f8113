#!/usr/bin/env python3
"""Low-precision inference (the MI355X counterpart of pyzoo/zoo/examples/vnni -- int8 VNNI
inference through OpenVINO on Xeon): a zoo ResNet is calibrated on a batch and served as its
static int8 twin (v_mfma_i32_16x16x64_i8) or OCP-fp8 twin (v_mfma_f32_16x16x128_f8f6f4) through
the InferenceModel replica pool; the example reports the agreement with the bf16 model."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401


def main(argv=None):
    ap = _common.add_common(argparse.ArgumentParser(description=__doc__.split("\n")[0]))
    ap.add_argument("--dtype", default="fp8", choices=["int8", "fp8"])
    ap.add_argument("--depth", type=int, default=50, choices=[18, 34, 50, 101, 152])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image-size", type=int, default=224)
    a = ap.parse_args(argv)
    import numpy as np
    import torch
    from zoo.models.image import resnet as R
    from zoo.pipeline.inference import InferenceModel
    torch.manual_seed(a.seed)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    m = getattr(R, "resnet%d" % a.depth)(num_classes=100).to(dev).eval()
    x = torch.randn(a.batch, 3, a.image_size, a.image_size)
    with torch.no_grad():
        ref = m(x.to(dev)).float().cpu().numpy()
    calib = torch.randn(a.batch, 3, a.image_size, a.image_size)
    im = InferenceModel(1, device=dev).load_module(m, blas=False, calib_data=calib, qdtype=a.dtype)
    out = im.predict(x)
    cos = float((out * ref).sum() / (np.linalg.norm(out) * np.linalg.norm(ref)))
    top1 = float((out.argmax(1) == ref.argmax(1)).mean())
    print("%s vs bf16: logit cosine %.4f, top-1 agreement %.2f" % (a.dtype, cos, top1))
    return {"cos": cos, "top1": top1}


if __name__ == "__main__":
    main()
