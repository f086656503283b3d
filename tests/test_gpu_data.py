"""Device image transform (csrc/image.hip capk_resize_normalize) vs the reference's own
pixel path: PIL crop + resize(BILINEAR) (torchvision's F.resized_crop / F.resize on PIL
images) -> flip -> ToTensor -> Normalize in torch fp32.  Bit-exact (torch.equal): the
kernel restates Pillow's fixed-point antialiased resampling.  Covers downscale and
upscale crops, both flips, the eval Resize + CenterCrop on landscape / portrait /
square images, bf16 output, and the DataLoader path end to end."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
cuda = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")

MEAN = torch.tensor([0.485, 0.456, 0.406], dtype=torch.float32)
STD = torch.tensor([0.229, 0.224, 0.225], dtype=torch.float32)


def _pil_ref(img, desc, S):
    from PIL import Image
    cy, cx, ch, cw, rh, rw, oy, ox, flip = desc
    im = Image.fromarray(img).crop((cx, cy, cx + cw, cy + ch)).resize((rw, rh), Image.BILINEAR)
    arr = np.asarray(im)[oy:oy + S, ox:ox + S]
    if flip:
        arr = arr[:, ::-1]
    t = torch.from_numpy(np.ascontiguousarray(arr)).permute(2, 0, 1).float().div(255)
    return t.sub(MEAN[:, None, None]).div(STD[:, None, None])


def _run(items, S, dtype=torch.float32):
    from capk import data as D
    batch = D.collate(items)
    return D.DeviceTransform("cuda", S, dtype=dtype)(batch)["image"].cpu()


def _item(img, desc):
    return {"image_u8": img, "desc": desc, "caption_tokens": torch.zeros(4, dtype=torch.long),
            "attention_mask": torch.zeros(4, dtype=torch.long)}


@cuda
def test_train_crops_bit_exact_vs_pil():
    from capk import data as D
    rng = np.random.default_rng(1)
    g = torch.Generator().manual_seed(2)
    S = 224
    items, refs = [], []
    for h, w in ((480, 640), (333, 500), (224, 224), (120, 90), (640, 427), (1000, 750)):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        for _ in range(3):
            d = D.train_desc(h, w, S, g)
            items.append(_item(img, d))
            refs.append(_pil_ref(img, d, S))
    got = _run(items, S)
    for k, r in enumerate(refs):
        assert torch.equal(got[k], r), (k, float((got[k] - r).abs().max()))


@cuda
def test_eval_resize_center_crop_bit_exact_vs_pil():
    from capk import data as D
    rng = np.random.default_rng(3)
    S = 224
    items, refs = [], []
    for h, w in ((480, 640), (640, 480), (224, 224), (300, 300), (150, 200), (2000, 1500)):
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        d = D.eval_desc(h, w, S)
        items.append(_item(img, d))
        refs.append(_pil_ref(img, d, S))
    got = _run(items, S)
    for k, r in enumerate(refs):
        assert torch.equal(got[k], r), (k, float((got[k] - r).abs().max()))
    got16 = _run(items, S, torch.bfloat16)
    assert torch.equal(got16.float(), torch.stack(refs).bfloat16().float())


@cuda
def test_coco_loader_end_to_end(tmp_path):
    """build_coco_dataloaders over a synthetic COCO tree: device batches equal the PIL path."""
    import json
    import os
    from PIL import Image
    from capk import config as C
    from capk import data as D
    from test_data import StubTokenizer
    os.makedirs(tmp_path / "tr")
    rng = np.random.default_rng(4)
    images, anns, arrays = [], [], {}
    for k, (h, w) in enumerate(((300, 400), (256, 256), (500, 333), (240, 320))):
        arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        Image.fromarray(arr).save(tmp_path / "tr" / f"{k}.png")
        arrays[k] = arr
        images.append({"id": k, "file_name": f"{k}.png"})
        anns += [{"image_id": k, "caption": f"caption {k} {c}"} for c in range(2)]
    with open(tmp_path / "a.json", "w") as f:
        json.dump({"images": images, "annotations": anns}, f)
    cfg = C.Config()
    cfg.data_root, cfg.train_json, cfg.val_json = str(tmp_path), "a.json", "a.json"
    cfg.train_image_dir = cfg.val_image_dir = "tr"
    cfg.num_workers = 0
    cfg.training.batch_size = 3
    cfg.inference.num_candidates = 2
    train, val, _ = D.build_coco_dataloaders(cfg, StubTokenizer(), device="cuda")
    n = 0
    for batch in train:
        assert batch["image"].shape[1:] == (3, 224, 224) and batch["image"].is_cuda
        assert batch["caption_tokens"].is_cuda
        n += batch["image"].shape[0]
    assert n == 8
    ds = train.loader.dataset
    b0 = D.collate([ds[0], ds[5]])
    got = D.DeviceTransform("cuda", 224)(b0)["image"].cpu()
    for k, idx in enumerate((0, 5)):
        assert torch.equal(got[k], _pil_ref(arrays[ds.examples[idx]["image_id"]], ds[idx]["desc"], 224))
    vb = next(iter(val))
    assert vb["image"].shape == (2, 3, 224, 224) and len(vb["captions"]) == 2


@cuda
def test_validate_over_coco_loaders(tmp_path):
    """CaptioningTrainer.validate over build_coco_dataloaders' eval loader: images with 1, 2
    and 3 reference captions in one batch (padded reference sets), CE on caption 0 and
    CIDEr-D of the greedy captions -- the path `--mode eval` and train() run."""
    import json
    import os
    from PIL import Image
    from capk import config as C
    from capk import data as D
    from capk.models import captioning_model as cm
    from capk.models import encoders as E
    from capk.train.trainer import CaptioningTrainer
    from test_data import StubTokenizer
    os.makedirs(tmp_path / "v")
    rng = np.random.default_rng(5)
    images, anns = [], []
    for k, (h, w) in enumerate(((240, 300), (256, 256), (230, 260))):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / "v" / f"{k}.png")
        images.append({"id": k, "file_name": f"{k}.png"})
        anns += [{"image_id": k, "caption": f"a caption of image {k} number {c}"} for c in range(k + 1)]
    with open(tmp_path / "a.json", "w") as f:
        json.dump({"images": images, "annotations": anns}, f)
    cfg = C.Config()
    cfg.data_root, cfg.train_json, cfg.val_json = str(tmp_path), "a.json", "a.json"
    cfg.train_image_dir = cfg.val_image_dir = "v"
    cfg.num_workers = 0
    cfg.inference.num_candidates = 3  # one eval batch holds all three images
    cfg.inference.max_length = 8
    cfg.model.encoder = C.EncoderConfig(encoder_type="vit", feature_dim=64)
    cfg.model.decoder = C.DecoderConfig(decoder_type="transformer", hidden_dim=64, num_layers=1, num_heads=2,
                                        max_length=12)
    cfg.model.vocab_size, cfg.model.pad_token_id, cfg.model.bos_token_id, cfg.model.eos_token_id = 1001, 0, 0, 0
    cfg.output_dir = cfg.checkpoint_dir = str(tmp_path / "out")
    arch = dict(hidden_size=64, num_hidden_layers=1, num_attention_heads=2, intermediate_size=128, image_size=224,
                patch_size=16, num_channels=3, layer_norm_eps=1e-12)
    orig = E.VIT_ARCHS["google/vit-base-patch16-224"]
    E.VIT_ARCHS["google/vit-base-patch16-224"] = arch
    try:
        torch.manual_seed(0)
        model = cm.ImageCaptioningModel(cfg)
    finally:
        E.VIT_ARCHS["google/vit-base-patch16-224"] = orig
    _, val, _ = D.build_coco_dataloaders(cfg, StubTokenizer(), device="cuda")
    vb = next(iter(val))
    assert vb["caption_tokens"].shape[:2] == (3, 3) and vb["num_references"].tolist() == [1, 2, 3]
    tr = CaptioningTrainer(cfg, model, None, val, StubTokenizer(), device="cuda", precision="fp32", total_steps=10)
    loss, metrics = tr.validate()
    assert np.isfinite(loss) and loss > 0 and np.isfinite(metrics["CIDEr"]) and metrics["CIDEr"] >= 0
