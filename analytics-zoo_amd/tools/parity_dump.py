#!/usr/bin/env python3
"""Dump the per-layer local parity rows (tools/layer_parity.py) of every ImageClassifier backbone
and both SSD detectors, training backward included, as JSON: the data behind the per-layer
bounds of tests/test_gpu_native_nets.py.
  python tools/parity_dump.py <out_dir> [name,name,...]"""
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import layer_parity  # noqa: E402

NETS = [("vgg-16", 224), ("alexnet", 227), ("squeezenet", 227), ("mobilenet", 224), ("mobilenet-v2", 224),
        ("inception-v1", 224), ("inception-v3", 299), ("densenet-161", 224)]


def main():
    out = sys.argv[1]
    only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None
    os.makedirs(out, exist_ok=True)
    from zoo.ops import _kern
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image import native_nets
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import softmax_cross_entropy
    init_nncontext("parity-dump")
    native_nets._dropout = lambda x, p, training: x
    dev = torch.device("cuda")
    for name, hw in NETS:
        if only and name not in only:
            continue
        _kern.reset_fault_counter()
        torch.manual_seed(0)
        net = build(name, 16)
        x = torch.randn(2, 3, hw, hw)
        y = torch.randint(0, 16, (2,))
        rows = layer_parity.run(copy.deepcopy(net).to(dev), copy.deepcopy(net), x.to(dev),
                                lambda o: softmax_cross_entropy(o, y.to(dev)), train=True)
        json.dump(rows, open(os.path.join(out, "parity_%s.json" % name), "w"), indent=0)
        print(name, len(rows), flush=True)
    from zoo.models.image.objectdetection.ssd import SSD, SSDMobileNet, MultiBoxLoss
    for mob in (False, True):
        if only and ("ssd-mobilenet" if mob else "ssd-vgg") not in only:
            continue
        _kern.reset_fault_counter()
        torch.manual_seed(0)
        model = SSDMobileNet(21) if mob else SSD(21)
        crit = MultiBoxLoss(21)
        gen = torch.Generator().manual_seed(0)
        x = torch.randn(2, 3, 300, 300)
        targets = []
        for _ in range(2):
            xy = torch.rand(3, 2, generator=gen) * 0.6
            wh = torch.rand(3, 2, generator=gen) * 0.3 + 0.05
            lab = torch.randint(1, 21, (3, 1), generator=gen).float()
            targets.append(torch.cat([lab, xy, xy + wh], 1))
        pri = model.priors.to(dev)
        tg = [t.to(dev) for t in targets]
        rows = layer_parity.run(copy.deepcopy(model).to(dev).train(), copy.deepcopy(model).train(), x.to(dev),
                                lambda o: crit(o[0].float(), o[1].float(), pri, tg), train=True)
        nm = "ssd-mobilenet" if mob else "ssd-vgg"
        json.dump(rows, open(os.path.join(out, "parity_%s.json" % nm), "w"), indent=0)
        print(nm, len(rows), flush=True)


if __name__ == "__main__":
    main()
