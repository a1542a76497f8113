"""Debug: first-step loss reproducibility across engines (ibo off/off/on), SGD lr 0.01."""
import copy, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "analytics-zoo_amd"))
import torch
from zoo.common.nncontext import init_nncontext
from zoo.models.image.resnet import resnet50
from zoo.ops import softmax_cross_entropy
from zoo.pipeline.api.keras.optimizers import SGD
from zoo.pipeline.engine import TrainingEngine
init_nncontext("dbg")
torch.manual_seed(0)
m = resnet50(num_classes=10)
gpu = torch.device("cuda")
x = torch.randn(16, 3, 64, 64, device=gpu)
y = torch.randint(0, 10, (16,), device=gpu)
for tag, ibo in (("off", "0"), ("off", "0"), ("on", "1"), ("on", "1")):
    os.environ["ZOO_OPTIM_IN_BWD"] = ibo
    eng = TrainingEngine(copy.deepcopy(m), softmax_cross_entropy, SGD(learningrate=0.01, momentum=0.9), bucket_mb=0.25,
                         hip_graph=False)
    with torch.no_grad():
        eng.model.train()
        l_fwd = float(softmax_cross_entropy(eng.model(x), y).float().item())
    ls = [float(eng.train_step(x, y).float().item()) for _ in range(4)]
    print(tag, eng.ibo, "fwd-only", round(l_fwd, 5), [round(v, 5) for v in ls], flush=True)
