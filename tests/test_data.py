"""Input pipeline host logic (capk/data.py; SURVEY §8f-2, reference src/data/dataset.py):
annotation processing (train: one example per caption, eval: grouped per image), the
tokenizer call contract, torchvision's RandomResizedCrop / Resize / CenterCrop parameter
rules, batch packing.  The pixel kernel is checked against PIL in tests/test_gpu_data.py."""
import json
import os

import numpy as np
import pytest
import torch

from capk import data as D


class _Enc:
    def __init__(self, ids, mask):
        self.input_ids, self.attention_mask = ids, mask


class StubTokenizer:
    """HF-tokenizer call contract used by the reference (dataset.py:118-124): one id per
    word, padded with pad_id to max_length, truncated."""
    pad_id = 0

    def __init__(self):
        self.calls = []

    def __call__(self, text, padding, truncation, max_length, return_tensors):
        self.calls.append((padding, truncation, max_length, return_tensors))
        ids = [(hash(w) % 1000) + 1 for w in text.split()][:max_length]
        mask = [1] * len(ids) + [0] * (max_length - len(ids))
        ids = ids + [self.pad_id] * (max_length - len(ids))
        return _Enc(torch.tensor([ids]), torch.tensor([mask]))


def _coco(tmp_path, sizes=((48, 64), (70, 30), (40, 40))):
    from PIL import Image
    os.makedirs(tmp_path / "imgs")
    rng = np.random.default_rng(0)
    images, anns = [], []
    for k, (h, w) in enumerate(sizes):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / "imgs" / f"{k}.png")
        images.append({"id": 100 + k, "file_name": f"{k}.png"})
        for c in range(2 + k):
            anns.append({"image_id": 100 + k, "caption": f"a picture number {k} caption {c}"})
    anns.append({"image_id": 999, "caption": "orphan caption"})  # skipped (dataset.py:67-69)
    with open(tmp_path / "ann.json", "w") as f:
        json.dump({"images": images, "annotations": anns}, f)
    return str(tmp_path)


def test_dataset_train_and_eval_items(tmp_path):
    root = _coco(tmp_path)
    tok = StubTokenizer()
    tr = D.COCOCaptionDataset(root, "ann.json", "imgs", tok, image_size=32, max_length=12, is_training=True)
    assert len(tr) == 2 + 3 + 4
    it = tr[0]
    assert it["image_u8"].shape == (48, 64, 3) and it["image_u8"].dtype == np.uint8
    assert it["caption_tokens"].shape == (12,) and it["attention_mask"].shape == (12,)
    assert tok.calls[-1] == ("max_length", True, 12, "pt")
    cy, cx, ch, cw, rh, rw, oy, ox, flip = it["desc"]
    assert 0 <= cy and cy + ch <= 48 and 0 <= cx and cx + cw <= 64 and (rh, rw, oy, ox) == (32, 32, 0, 0)
    assert it["desc"] == tr[0]["desc"]  # deterministic per (seed, epoch, index)
    ev = D.COCOCaptionDataset(root, "ann.json", "imgs", tok, image_size=32, max_length=12, is_training=False)
    assert len(ev) == 3
    e2 = ev[2]
    assert e2["caption_tokens"].shape == (4, 12) and len(e2["captions"]) == 4 and e2["image_id"] == 102
    assert e2["desc"] == (0, 0, 40, 40, 32, 32, 0, 0, 0)


def test_random_resized_crop_params_rules():
    g = torch.Generator().manual_seed(1)
    for _ in range(300):
        h, w = int(torch.randint(20, 900, (1,))), int(torch.randint(20, 900, (1,)))
        i, j, ch, cw = D.random_resized_crop_params(h, w, g)
        assert 0 <= i and i + ch <= h and 0 <= j and j + cw <= w and ch > 0 and cw > 0
    # fallback: an extreme aspect ratio never satisfies the 10 draws -> ratio-clamped center crop
    i, j, ch, cw = D.random_resized_crop_params(10, 2000, torch.Generator().manual_seed(0), scale=(0.99, 1.0))
    assert (ch, cw) == (10, 13) and (i, j) == (0, (2000 - 13) // 2)


def test_resize_and_center_crop_sizes():
    assert D.resize_shorter(480, 640, 224) == (224, int(224 * 640 / 480))
    assert D.resize_shorter(640, 480, 224) == (int(224 * 640 / 480), 224)
    assert D.center_crop_origin(224, 298, 224) == (0, 37)
    assert D.eval_desc(480, 640, 224) == (0, 0, 480, 640, 224, 298, 0, 37, 0)


def test_collate_packs_images(tmp_path):
    root = _coco(tmp_path)
    tr = D.COCOCaptionDataset(root, "ann.json", "imgs", StubTokenizer(), image_size=32, max_length=8)
    items = [tr[k] for k in (0, 3, 6)]
    b = D.collate(items)
    import ctypes
    descs = (D._ImgDesc * 3).from_buffer_copy(bytes(b["image_desc"].numpy()))
    buf = b["images_packed"].numpy()
    for it, d in zip(items, descs):
        img = it["image_u8"]
        assert (d.H, d.W) == img.shape[:2] and d.offset % 16 == 0
        assert np.array_equal(buf[d.offset:d.offset + img.nbytes].reshape(img.shape), img)
    assert b["caption_tokens"].shape == (3, 8)
    assert ctypes.sizeof(D._ImgDesc) == 56


def test_eval_collate_pads_reference_sets(tmp_path):
    """Eval items carry 2, 3 and 4 references: the batch stacks them to [3, 4, L] with pad
    rows (the tokenizer's pad id, mask 0) and records each image's own count."""
    root = _coco(tmp_path)
    ev = D.COCOCaptionDataset(root, "ann.json", "imgs", StubTokenizer(), image_size=32, max_length=6,
                              is_training=False)
    items = [ev[k] for k in range(3)]
    b = D.collate(items)
    assert b["caption_tokens"].shape == (3, 4, 6) and b["attention_mask"].shape == (3, 4, 6)
    assert b["num_references"].tolist() == [2, 3, 4]
    for k, it in enumerate(items):
        n = it["caption_tokens"].shape[0]
        assert torch.equal(b["caption_tokens"][k, :n], it["caption_tokens"])
        assert bool((b["caption_tokens"][k, n:] == StubTokenizer.pad_id).all())
        assert int(b["attention_mask"][k, n:].sum()) == 0


def test_epoch_sampler_changes_augmentation_per_epoch(tmp_path):
    """EpochSampler: a fresh permutation per pass, each index tagged with its epoch, so the
    crop / flip draws differ between epochs and repeat for the same (epoch, index) -- also
    inside persistent DataLoader workers, which never see set_epoch."""
    root = _coco(tmp_path)
    tr = D.COCOCaptionDataset(root, "ann.json", "imgs", StubTokenizer(), image_size=32, max_length=8)
    s = D.EpochSampler(len(tr), seed=3)
    e0, e1 = list(s), list(s)
    assert sorted(i for i, _ in e0) == list(range(len(tr))) and {e for _, e in e0} == {0} and {e for _, e in e1} == {1}
    assert [i for i, _ in e0] != [i for i, _ in e1]
    descs = lambda ep: [tr[(i, ep)]["desc"] for i in range(len(tr))]
    assert descs(0) != descs(1) and descs(1) == descs(1)
    s.set_epoch(5)
    assert {e for _, e in s} == {5}
    loader = torch.utils.data.DataLoader(tr, batch_size=len(tr), sampler=D.EpochSampler(len(tr), 3),
                                         collate_fn=lambda it: [x["desc"] for x in it], num_workers=1,
                                         persistent_workers=True)
    a, b = next(iter(loader)), next(iter(loader))
    assert sorted(a) != sorted(b)  # second pass = epoch 1: different crops
