"""Per-block divergence of the capk ResNet-101 (fp32 and bf16) from the CPU oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "image-captioning-ml-project_amd")]
import torch
import torch.nn.functional as F
import capk
from capk.models import resnet as R
from oracle import encoders as oenc


def rel(a, b):
    return float((a.float().cpu() - b.float()).norm() / b.float().norm())


for prec in ("fp32", "bf16"):
    torch.manual_seed(11)
    m = R.CapkResNetModel(R.RESNET_ARCHS["microsoft/resnet-101"])
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    capk.prepare(m, "cuda", prec)
    m.train()
    B = 2
    images = torch.randn(B, 3, 224, 224)
    st = {k: v.clone() for k, v in sd.items()}
    with torch.no_grad():
        x, H, W = m.embedder(images.cuda())
        r = oenc._conv_bn(sd, "embedder.embedder.", images, 2, True, True, st)
        r = F.max_pool2d(r, 3, 2, 1)
        print(prec, "stem", rel(x, r.permute(0, 2, 3, 1).reshape(-1, r.shape[1])))
        for si, depth in enumerate([3, 4, 23, 3]):
            for li in range(depth):
                layer = m.encoder.stages[si].layers[li]
                x, H, W = layer(x, B, H, W)
                pre = f"encoder.stages.{si}.layers.{li}."
                stride = (2 if si > 0 else 1) if li == 0 else 1
                h = oenc._conv_bn(sd, pre + "layer.0.", r, 1, True, True, st)
                h = oenc._conv_bn(sd, pre + "layer.1.", h, stride, True, True, st)
                h = oenc._conv_bn(sd, pre + "layer.2.", h, 1, True, False, st)
                rr = oenc._conv_bn(sd, pre + "shortcut.", r, stride, True, False, st) if pre + "shortcut.convolution.weight" in sd else r
                r = F.relu(h + rr)
                print(prec, si, li, "rel", round(rel(x, r.permute(0, 2, 3, 1).reshape(-1, r.shape[1])), 5),
                      "norm", round(float(r.norm()), 1))
