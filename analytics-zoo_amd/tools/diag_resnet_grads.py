"""Diagnose ResNet gradient agreement: GPU (bf16 native) vs CPU fp32 vs CPU bf16-rounded activations."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from zoo.models.image.resnet import ResNet, Bottleneck
from zoo.ops import softmax_cross_entropy

torch.manual_seed(0)
mk = lambda: ResNet(Bottleneck, [1, 1, 1, 1], num_classes=16, width=16)
m32 = mk(); mbf = mk(); mg = mk()
mbf.load_state_dict(m32.state_dict()); mg.load_state_dict(m32.state_dict())
x = torch.randn(8, 3, 128, 128); y = torch.randint(0, 16, (8,))
softmax_cross_entropy(m32(x), y).backward()
# bf16 CPU: feed NHWC bf16 so every conv_bn_act output is rounded to bf16
xb = F.pad(x.permute(0, 2, 3, 1), (0, 1)).bfloat16()
softmax_cross_entropy(mbf(xb), y).backward()
mg = mg.cuda()
softmax_cross_entropy(mg(x.cuda()), y.cuda()).backward()
p32 = dict(m32.named_parameters()); pbf = dict(mbf.named_parameters())
cos = lambda a, b: F.cosine_similarity(a.flatten().double(), b.flatten().double(), dim=0).item()
for n, p in mg.named_parameters():
    print("%-32s gpu~fp32 %.4f  cpubf16~fp32 %.4f  gpu~cpubf16 %.4f" % (n, cos(p.grad.cpu(), p32[n].grad),
          cos(pbf[n].grad, p32[n].grad), cos(p.grad.cpu(), pbf[n].grad)))
