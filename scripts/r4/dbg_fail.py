"""Debug the round-4 full-suite failures: mobilenet-v2 layer parity rows, train_briefly accuracy."""
import copy, os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd", "tools"))
import torch
from zoo.common.nncontext import init_nncontext
init_nncontext("dbg")
gpu = torch.device("cuda")
what = sys.argv[1]
if what == "mnv2":
    import layer_parity as lp
    from zoo.models.image import native_nets
    from zoo.models.image.imageclassification.nets import build
    from zoo.ops import softmax_cross_entropy
    native_nets._dropout = lambda x, p, training: x
    torch.manual_seed(0)
    net = build("mobilenet-v2", 16)
    cpu = copy.deepcopy(net)
    g = copy.deepcopy(net).to(gpu)
    x = torch.randn(2, 3, 224, 224)
    y = torch.randint(0, 16, (2,))
    rows = lp.run(g, cpu, x.to(gpu), lambda o: softmax_cross_entropy(o, y.to(gpu)), train=True)
    for r in rows:
        if "error" in r or r.get("fwd", 0) > 0.02:
            print(json.dumps(r)[:400])
else:
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    from zoo.utils.synthetic import class_templates, sample
    steps, lr, batch, noise = int(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
    torch.manual_seed(0)
    m = resnet50(num_classes=16).to(gpu)
    T = class_templates(16, 128, device=gpu)
    eng = TrainingEngine(m, softmax_cross_entropy, SGD(learningrate=lr, momentum=0.9))
    ls = []
    for s_ in range(steps):
        x, y = sample(T, batch, seed=200003 + s_, noise=noise)
        ls.append(float(eng.train_step(x, y).float().item()))
    eng.flat.detach()
    x, y = sample(T, 128, seed=999, noise=noise)
    with torch.no_grad():
        m.train()
        acc_tr = (m(x).float().argmax(1) == y).float().mean().item()
        m.eval()
        acc_ev = (m(x).float().argmax(1) == y).float().mean().item()
    print(what, "steps", steps, "lr", lr, "batch", batch, "noise", noise, "loss", [round(v, 3) for v in ls[::max(1, steps // 8)]],
          "acc train-mode", acc_tr, "acc eval", acc_ev, flush=True)
