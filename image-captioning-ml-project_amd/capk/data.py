"""COCO caption input pipeline — mirrors src/data/dataset.py:12-177,390-472
and the transforms of src/main.py:139-153, with the pixel work on the GPU.

* ``COCOCaptionDataset`` — the reference's dataset (same annotation processing, train =
  one example per caption, eval = one example per image with all its captions; the
  tokenizer is called exactly as the reference calls it: ``padding='max_length'``,
  ``truncation=True``, ``max_length``).  ``__getitem__`` returns the decoded image as
  uint8 RGB ``[H, W, 3]`` (PIL, as the reference) plus the crop box / flip of the
  transform, sampled here with torchvision's algorithms (restated below) — the resampling
  itself is deferred to the device.
* ``collate`` packs a batch's uint8 images into one pinned byte buffer + per-image
  descriptors; ``DeviceTransform`` uploads it once (non-blocking) and runs
  ``capk_resize_normalize`` (csrc/image.hip): crop + Pillow-exact antialiased bilinear
  resize + flip + ToTensor + Normalize in one kernel, bit-identical to PIL + torchvision.
  Eval batches stack every image's reference set into ``[B, N, L]`` (pad rows past the
  image's own ``num_references``).
* ``build_coco_dataloaders(config, tokenizer, ...)`` — the reference's factory
  (dataset.py:390-472; curriculum sampling is out of scope) returning loaders whose batches
  are already on the device: ``{"image": [B,3,S,S], "caption_tokens", "attention_mask",
  ...}``.
"""
import ctypes
import json
import math
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from . import _lib
from ._lib import check

IMAGENET_MEAN = (0.485, 0.456, 0.406)  # main.py:144-145
IMAGENET_STD = (0.229, 0.224, 0.225)
MAX_DOWNSCALE = 31  # csrc/image.hip RS_KMAX taps


# ---------------------------------------------------------- transform params ----
def random_resized_crop_params(height, width, gen, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0)):
    """torchvision.transforms.RandomResizedCrop.get_params restated (same draws, same
    fallback): returns (top, left, h, w) of the crop box."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=gen).item()
        aspect_ratio = torch.exp(torch.empty(1).uniform_(float(log_ratio[0]), float(log_ratio[1]),
                                                         generator=gen)).item()
        w = int(round(math.sqrt(target_area * aspect_ratio)))
        h = int(round(math.sqrt(target_area / aspect_ratio)))
        if 0 < w <= width and 0 < h <= height:
            i = int(torch.randint(0, height - h + 1, size=(1,), generator=gen).item())
            j = int(torch.randint(0, width - w + 1, size=(1,), generator=gen).item())
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


def resize_shorter(height, width, size):
    """torchvision Resize(int) output size (shorter side -> size, the other truncated)."""
    if width <= height:
        return int(size * height / width), size
    return size, int(size * width / height)


def center_crop_origin(height, width, size):
    """torchvision CenterCrop origin (top, left) of a size x size window."""
    return int(round((height - size) / 2.0)), int(round((width - size) / 2.0))


def train_desc(h, w, size, gen, flip_p=0.5):
    """RandomResizedCrop(size) -> RandomHorizontalFlip(flip_p): (cy, cx, ch, cw, rh, rw, oy, ox, flip)."""
    i, j, ch, cw = random_resized_crop_params(h, w, gen)
    flip = int(torch.rand(1, generator=gen).item() < flip_p)
    return (i, j, ch, cw, size, size, 0, 0, flip)


def eval_desc(h, w, size):
    """Resize(size) -> CenterCrop(size)."""
    rh, rw = resize_shorter(h, w, size)
    oy, ox = center_crop_origin(rh, rw, size)
    return (0, 0, h, w, rh, rw, oy, ox, 0)


class _ImgDesc(ctypes.Structure):  # csrc/image.hip ImgDesc
    _fields_ = [("offset", ctypes.c_int64), ("H", ctypes.c_int), ("W", ctypes.c_int), ("cy", ctypes.c_int),
                ("cx", ctypes.c_int), ("ch", ctypes.c_int), ("cw", ctypes.c_int), ("rh", ctypes.c_int),
                ("rw", ctypes.c_int), ("oy", ctypes.c_int), ("ox", ctypes.c_int), ("flip", ctypes.c_int)]


# ------------------------------------------------------------------ dataset ----
def decode_rgb(path):
    """Image.open(path).convert('RGB') as uint8 [H, W, 3] (dataset.py:110)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


class COCOCaptionDataset(Dataset):
    """src/data/dataset.py:12-177 with the transform split into host params + device pixels."""

    def __init__(self, root_dir, annotation_file, image_dir, tokenizer, image_size=224, max_length=50,
                 is_training=True, seed=0):
        self.root_dir = root_dir
        self.image_dir = os.path.join(root_dir, image_dir)
        self.annotation_path = os.path.join(root_dir, annotation_file)
        self.tokenizer = tokenizer
        self.image_size = image_size
        self.max_length = max_length
        self.is_training = is_training
        self.seed = seed
        self.epoch = 0
        self.pad_token_id = int(getattr(tokenizer, "pad_token_id", None) or 0)
        with open(self.annotation_path, "r") as f:
            self.annotations = json.load(f)
        self._process_annotations()

    def _process_annotations(self):  # dataset.py:54-100
        fname = {im["id"]: im["file_name"] for im in self.annotations["images"]}
        self.examples = [{"image_id": a["image_id"], "filename": fname[a["image_id"]], "caption": a["caption"]}
                         for a in self.annotations["annotations"] if a["image_id"] in fname]
        if not self.is_training:
            grouped = {}
            for ex in self.examples:
                g = grouped.setdefault(ex["image_id"], {"filename": ex["filename"], "captions": []})
                g["captions"].append(ex["caption"])
            self.examples = [{"image_id": k, "filename": v["filename"], "captions": v["captions"]}
                             for k, v in grouped.items()]

    def __len__(self):
        return len(self.examples)

    def _tok(self, caption):
        enc = self.tokenizer(caption, padding="max_length", truncation=True, max_length=self.max_length,
                             return_tensors="pt")
        return enc.input_ids.squeeze(0), enc.attention_mask.squeeze(0)

    def set_epoch(self, epoch):
        """Epoch mixed into the crop / flip draws of a plain integer index (EpochSampler
        passes (index, epoch) pairs instead, which also reach persistent workers)."""
        self.epoch = int(epoch)

    def __getitem__(self, idx):
        epoch = self.epoch
        if isinstance(idx, tuple):  # (index, epoch) from EpochSampler
            idx, epoch = idx
        ex = self.examples[idx]
        img = decode_rgb(os.path.join(self.image_dir, ex["filename"]))
        h, w = img.shape[:2]
        if self.is_training:
            # torchvision draws fresh crop / flip parameters on every access; here they are a
            # function of (seed, epoch, index): new every epoch, reproducible per run
            gen = torch.Generator().manual_seed((self.seed * 1_000_003 + epoch) * 10_000_019 + idx)
            desc = train_desc(h, w, self.image_size, gen)
            ids, mask = self._tok(ex["caption"])
            return {"image_u8": img, "desc": desc, "caption_tokens": ids, "attention_mask": mask,
                    "caption": ex["caption"]}
        desc = eval_desc(h, w, self.image_size)
        toks = [self._tok(c) for c in ex["captions"]]
        if toks:
            ids = torch.stack([t[0] for t in toks])
            mask = torch.stack([t[1] for t in toks])
        else:  # dataset.py:166-171
            ids = torch.zeros((1, self.max_length), dtype=torch.long)
            mask = torch.zeros((1, self.max_length), dtype=torch.long)
        return {"image_u8": img, "desc": desc, "caption_tokens": ids, "attention_mask": mask,
                "captions": ex["captions"], "image_id": ex["image_id"], "pad_token_id": self.pad_token_id}


class EpochSampler(torch.utils.data.Sampler):
    """shuffle=True of the reference's train loader (dataset.py:436-444): a fresh permutation
    per pass, each index tagged with the pass number, so the dataset's crop / flip draws
    change every epoch even inside persistent workers (which never see set_epoch)."""

    def __init__(self, n, seed=0):
        self.n, self.seed, self.epoch = int(n), int(seed), -1

    def set_epoch(self, epoch):
        self.epoch = int(epoch) - 1  # the next __iter__ runs epoch `epoch`

    def __len__(self):
        return self.n

    def __iter__(self):
        self.epoch += 1
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + self.epoch)
        ep = self.epoch
        return iter([(i, ep) for i in torch.randperm(self.n, generator=g).tolist()])


def _stack_padded(rows, fill):
    """[N_i, L] tensors -> [B, max N_i, L]; missing rows filled with `fill`."""
    n = max(r.shape[0] for r in rows)
    out = torch.full((len(rows), n, rows[0].shape[1]), fill, dtype=rows[0].dtype)
    for b, r in enumerate(rows):
        out[b, :r.shape[0]] = r
    return out


def collate(items):
    """Packs uint8 images into one pinned buffer + an ImgDesc array; stacks the tokens."""
    offs, total = [], 0
    for it in items:
        offs.append(total)
        total += (it["image_u8"].nbytes + 15) // 16 * 16
    buf = torch.empty(max(total, 16), dtype=torch.uint8)  # pinned by the DataLoader (main process)
    npbuf = buf.numpy()
    descs = (_ImgDesc * len(items))()
    for k, (it, off) in enumerate(zip(items, offs)):
        img = it["image_u8"]
        h, w = img.shape[:2]
        npbuf[off:off + img.nbytes] = img.reshape(-1)
        cy, cx, ch, cw, rh, rw, oy, ox, flip = it["desc"]
        if ch > MAX_DOWNSCALE * rh or cw > MAX_DOWNSCALE * rw:
            raise ValueError(f"capk data: downscale {ch}x{cw} -> {rh}x{rw} exceeds {MAX_DOWNSCALE}x")
        descs[k] = _ImgDesc(off, h, w, cy, cx, ch, cw, rh, rw, oy, ox, flip)
    out = {"images_packed": buf, "image_desc": torch.frombuffer(bytearray(descs), dtype=torch.uint8).clone()}
    if items[0]["caption_tokens"].dim() == 1:
        out["caption_tokens"] = torch.stack([it["caption_tokens"] for it in items])
        out["attention_mask"] = torch.stack([it["attention_mask"] for it in items])
    else:  # eval: every image's reference set, padded to the batch's largest with pad rows
        pad = items[0].get("pad_token_id", 0)
        out["caption_tokens"] = _stack_padded([it["caption_tokens"] for it in items], pad)
        out["attention_mask"] = _stack_padded([it["attention_mask"] for it in items], 0)
        out["num_references"] = torch.tensor([it["caption_tokens"].shape[0] for it in items], dtype=torch.long)
    for key in ("caption", "captions", "image_id"):
        if key in items[0]:
            out[key] = [it[key] for it in items]
    return out


class DeviceTransform:
    """Uploads a collated batch (pinned, non-blocking) and produces the normalised
    [B, 3, S, S] images on the device with one capk_resize_normalize launch."""

    def __init__(self, device, image_size=224, mean=IMAGENET_MEAN, std=IMAGENET_STD, dtype=torch.float32):
        self.device = torch.device(device)
        self.size = image_size
        self.mean = (ctypes.c_float * 3)(*mean)
        self.std = (ctypes.c_float * 3)(*std)
        self.dtype = dtype

    def __call__(self, batch):
        L = _lib.load()
        if ctypes.sizeof(_ImgDesc) != L.capk_image_desc_bytes():
            raise _lib.CapkError("capk data: ImgDesc layout differs from libcapk's")
        images = batch["images_packed"].to(self.device, non_blocking=True)
        desc = batch["image_desc"].to(self.device, non_blocking=True)
        B = desc.numel() // ctypes.sizeof(_ImgDesc)
        out = torch.empty(B, 3, self.size, self.size, dtype=self.dtype, device=self.device)
        check(L.capk_resize_normalize(_lib.F32 if self.dtype == torch.float32 else _lib.BF16, B, self.size,
                                      images.data_ptr(), desc.data_ptr(), ctypes.cast(self.mean, ctypes.c_void_p),
                                      ctypes.cast(self.std, ctypes.c_void_p), out.data_ptr(),
                                      torch.cuda.current_stream(self.device).cuda_stream), "capk_resize_normalize")
        res = {k: v for k, v in batch.items() if k not in ("images_packed", "image_desc")}
        res["image"] = out
        for k in ("caption_tokens", "attention_mask"):
            if torch.is_tensor(res.get(k)):
                res[k] = res[k].to(self.device, non_blocking=True)
        return res


class DeviceLoader:
    """A DataLoader whose batches come out transformed on the device."""

    def __init__(self, loader, transform):
        self.loader, self.transform = loader, transform

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield self.transform(batch)


def build_coco_dataloaders(config, tokenizer, device=None, use_curriculum=None):
    """dataset.py:390-472 (curriculum sampling out of scope): (train_loader, val_loader, None)."""
    if use_curriculum or (use_curriculum is None and getattr(config.training, "use_curriculum", False)):
        raise NotImplementedError("capk data: curriculum sampling is out of scope (SURVEY §2)")
    device = device or (f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu")
    ml = config.model.decoder.max_length
    train_ds = COCOCaptionDataset(config.data_root, config.train_json, config.train_image_dir, tokenizer,
                                  config.image_size, ml, is_training=True, seed=config.seed)
    val_ds = COCOCaptionDataset(config.data_root, config.val_json, config.val_image_dir, tokenizer,
                                config.image_size, ml, is_training=False, seed=config.seed)
    kw = dict(num_workers=config.num_workers, collate_fn=collate, pin_memory=torch.cuda.is_available(),
              persistent_workers=config.num_workers > 0)
    train = DataLoader(train_ds, batch_size=config.training.batch_size,
                       sampler=EpochSampler(len(train_ds), config.seed), **kw)
    val = DataLoader(val_ds, batch_size=config.inference.num_candidates, shuffle=False, **kw)
    tf = DeviceTransform(device, config.image_size)
    return DeviceLoader(train, tf), DeviceLoader(val, tf), None


def load_image(path, image_size=224, device="cuda"):
    """Demo-mode image (main.py:270-343: eval transform) -> [3, S, S] on the device."""
    img = decode_rgb(path)
    h, w = img.shape[:2]
    batch = collate([{"image_u8": img, "desc": eval_desc(h, w, image_size),
                      "caption_tokens": torch.zeros(1, dtype=torch.long),
                      "attention_mask": torch.zeros(1, dtype=torch.long)}])
    return DeviceTransform(device, image_size)(batch)["image"][0]
