"""Legacy Show-Attend-Tell path on libcapk kernels.

Drop-in for the reference's root-level scripts:

  ``Encoder()``                      models/encoder.py:5-16   torchvision resnet101 trunk
                                                              + AdaptiveAvgPool2d(14) + permute
  ``Decoder(vocab_size, use_bert, device)``  models/decoder.py:9-176  LSTMCell decoder with
                                                              gated ReLU soft attention
  ``LegacyCaptionLoss``              train.py:92-101          packed CE + doubly stochastic
                                                              attention regulariser
  ``LegacyAdam``                     train.py:66-67,105-112   grad clamp +-5, Adam 4e-4
  ``train_step`` / ``decay_lr``      train.py:76-123          one batch of train()

Parameter and buffer names match the reference modules (``resnet.{0,1,4..7}...`` with
torchvision's Bottleneck names; ``enc_att``, ``dec_att``, ``att``, ``decode_step``
(nn.LSTMCell), ``h_lin``, ``c_lin``, ``f_beta``, ``fc``, ``embedding``).  Restatements
(SURVEY §0.1 D12): ``vocab_size`` is an int (a Vocabulary is accepted and its length
used), ``use_bert=False`` (BERT embeddings need the network: out of scope).

The decoder keeps the reference's shrinking batch: step t runs on the first
``batch_size_t = #{dec_len > t}`` rows (captions sorted by length, data_loader.py:65-76).
The encoder-side attention projection ``enc_att(encoder_out)`` does not depend on t, so
it is computed once per image instead of once per step (same values); the embedding
part of the LSTM input projection and the output layer run as one GEMM over all steps.
"""
import torch
import torch.nn as nn

from . import ops
from ._lib import ACT_SIGMOID
from .models.common import G, CapkModule, W, next_seed
from .models.resnet import BottleneckBlock, kernel_layout, stem_forward
from .models.transformer import _pad64

PAD, START, END, UNK = 0, 1, 2, 3  # models/constants.py
ATT_RELU = 1                         # additive-attention energy: relu (decoder.py:145-146)


# ---------------------------------------------------------------- encoder ----
class Bottleneck(BottleneckBlock):
    """torchvision.models.resnet.Bottleneck (expansion 4, stride on conv2: v1.5)."""

    def __init__(self, inplanes, planes, stride=1, downsample=False):
        super().__init__()
        self.conv1 = kernel_layout(nn.Conv2d(inplanes, planes, 1, bias=False))
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = kernel_layout(nn.Conv2d(planes, planes, 3, stride, 1, bias=False))
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = kernel_layout(nn.Conv2d(planes, planes * 4, 1, bias=False))
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = (nn.Sequential(kernel_layout(nn.Conv2d(inplanes, planes * 4, 1, stride, bias=False)),
                                         nn.BatchNorm2d(planes * 4)) if downsample else None)
        self.stride = stride

    def units(self):
        return [(self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)]

    def shortcut_units(self):
        return None if self.downsample is None else (self.downsample[0], self.downsample[1])


def _make_layer(inplanes, planes, blocks, stride):
    layers = [Bottleneck(inplanes, planes, stride, downsample=(stride != 1 or inplanes != planes * 4))]
    layers += [Bottleneck(planes * 4, planes) for _ in range(1, blocks)]
    return nn.Sequential(*layers)


class _AdaptivePoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, B, H, W, OH, OW):
        C = x.shape[1]
        ctx.geo = (B, H, W, C, OH, OW)
        return ops.avgpool_fwd(x, B, H, W, C, OH, OW)

    @staticmethod
    def backward(ctx, dy):
        B, H, W, C, OH, OW = ctx.geo
        return ops.avgpool_bwd(dy.contiguous(), B, H, W, C, OH, OW), None, None, None, None, None


class Encoder(CapkModule):
    """models/encoder.py:5-16: ``nn.Sequential(*list(resnet101.children())[:-2])`` then
    AdaptiveAvgPool2d((14, 14)) and permute(0, 2, 3, 1) -> [B, 14, 14, 2048].  Channels-last
    activations make the permute free.  Weights: torchvision's init (kaiming-normal fan_out
    convs, BN 1/0) — ``pretrained=True`` needs the network; load a checkpoint instead."""

    def __init__(self, layers=(3, 4, 23, 3), encoded_size=14):
        super().__init__()
        conv1 = kernel_layout(nn.Conv2d(3, 64, 7, 2, 3, bias=False))
        self.resnet = nn.Sequential(conv1, nn.BatchNorm2d(64), nn.ReLU(inplace=True), nn.MaxPool2d(3, 2, 1),
                                    _make_layer(64, 64, layers[0], 1), _make_layer(256, 128, layers[1], 2),
                                    _make_layer(512, 256, layers[2], 2), _make_layer(1024, 512, layers[3], 2))
        self.adaptive_pool = nn.AdaptiveAvgPool2d((encoded_size, encoded_size))
        self.encoded_size = encoded_size
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def stem_units(self):
        return self.resnet[0], self.resnet[1]

    def blocks(self):
        for stage in list(self.resnet)[4:]:
            for blk in stage:
                yield blk

    def forward(self, images):
        B = images.shape[0]
        x, H, W = stem_forward(self, images)
        for blk in self.blocks():
            x, H, W = blk(x, B, H, W)
        E = self.encoded_size
        out = _AdaptivePoolFn.apply(x, B, H, W, E, E)
        return out.view(B, E, E, x.shape[1])


# ---------------------------------------------------------------- decoder ----
class _LSTMCellParams(nn.Module):
    """nn.LSTMCell's parameter names and init (uniform(-1/sqrt(H), 1/sqrt(H)))."""

    def __init__(self, input_size, hidden_size):
        super().__init__()
        ref = nn.LSTMCell(input_size, hidden_size, bias=True)
        self.weight_ih, self.weight_hh = ref.weight_ih, ref.weight_hh
        self.bias_ih, self.bias_hh = ref.bias_ih, ref.bias_hh
        self.input_size, self.hidden_size = input_size, hidden_size


class Decoder(CapkModule):
    """models/decoder.py:9-176 (use_bert=False)."""

    def __init__(self, vocab_size, use_bert=False, device=None):
        super().__init__()
        if use_bert:
            raise NotImplementedError("capk legacy Decoder: BERT embeddings need from_pretrained (network); "
                                      "SURVEY §0.1 D12 restates the path with use_bert=False")
        if not isinstance(vocab_size, int):
            vocab_size = len(vocab_size)  # D12: the reference passes its Vocabulary object
        self.encoder_dim, self.attention_dim = 2048, 512
        self.embed_dim, self.decoder_dim = 512, 512
        self.use_bert = False
        self.device = device
        self.vocab_size = vocab_size
        self.vocab_pad = _pad64(vocab_size)
        self.enc_att = nn.Linear(2048, 512)
        self.dec_att = nn.Linear(512, 512)
        self.att = nn.Linear(512, 1)
        self.relu = nn.ReLU()
        self.softmax = nn.Softmax(dim=1)
        self.dropout = nn.Dropout(p=0.5)
        self.decode_step = _LSTMCellParams(self.embed_dim + self.encoder_dim, self.decoder_dim)
        self.h_lin = nn.Linear(self.encoder_dim, self.decoder_dim)
        self.c_lin = nn.Linear(self.encoder_dim, self.decoder_dim)
        self.f_beta = nn.Linear(self.decoder_dim, self.encoder_dim)
        self.sigmoid = nn.Sigmoid()
        self.fc = nn.Linear(self.decoder_dim, vocab_size)
        self.fc.bias.data.fill_(0)
        self.fc.weight.data.uniform_(-0.1, 0.1)
        self.fc.weight._capk_pad_rows = self.vocab_pad
        self.fc.bias._capk_pad_rows = self.vocab_pad
        self.embedding = nn.Embedding(vocab_size, self.embed_dim)
        self.embedding.weight.data.uniform_(-0.1, 0.1)

    def forward(self, encoder_out, encoded_captions, caption_lengths):
        """-> (predictions [B, max_dec_len, V], encoded_captions, dec_len, alphas [B, max_dec_len, P])."""
        lengths = [int(x) for x in caption_lengths]
        dec_len = [x - 1 for x in lengths]
        B = encoder_out.shape[0]
        enc = encoder_out.reshape(B, -1, encoder_out.shape[-1])
        preds, alphas = _LegacyDecoderFn.apply(enc, encoded_captions, self.fc.weight, self, tuple(dec_len))
        return preds, encoded_captions, dec_len, alphas


def _pad_w(lin, dt):
    return lin.weight._capk_pad_bf16 if dt == torch.bfloat16 else lin.weight._capk_pad_master


class _LegacyDecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, enc, captions, anchor, m, dec_len):
        ctx.set_materialize_grads(False)
        dt = m.cdtype
        dev = enc.device
        if enc.dtype != dt:
            raise TypeError(f"capk legacy Decoder: encoder_out dtype {enc.dtype} != compute dtype {dt}")
        B, S, De = enc.shape
        A, D, E = m.attention_dim, m.decoder_dim, m.embed_dim
        V, Vp = m.vocab_size, m.vocab_pad
        Tm = max(dec_len)
        bts = [sum(1 for x in dec_len if x > t) for t in range(Tm)]
        eff = [sum(1 for t in range(Tm) if b < bts[t]) for b in range(B)]  # active steps of row b
        enc = enc.contiguous()
        enc2 = enc.view(B * S, De)
        cs = m.decode_step
        # init hidden state with the average pixel (decoder.py:127-129)
        avg = ops.avgpool_fwd(enc2, B, S, 1, De, 1, 1)
        h0 = ops.linear(avg, W(m.h_lin.weight, dt), m.h_lin.bias.detach())
        c0 = ops.linear(avg, W(m.c_lin.weight, dt), m.c_lin.bias.detach(), out_dtype=torch.float32)
        Hs = torch.zeros(Tm + 1, B, D, dtype=dt, device=dev)
        Cs = torch.zeros(Tm + 1, B, D, dtype=torch.float32, device=dev)
        ops.copy_rows(h0, Hs[0])
        ops.copy_rows(c0, Cs[0])
        # hoisted: enc_att(encoder_out) (decoder.py:143, same for every t) and the embedding
        # part of the LSTM input projection for every step (t-major rows t*B + b)
        kp = ops.linear(enc2, W(m.enc_att.weight, dt), m.enc_att.bias.detach()).view(B, S, A)
        ids_t = captions[:, :Tm].t().contiguous()
        emb = ops.embedding_fwd(ids_t, m.embedding.weight.detach(), None, 0, dt)  # [Tm*B, E]
        w_ih = W(cs.weight_ih, dt)
        pre = ops.linear(emb, w_ih[:, :E], cs.bias_ih.detach())  # [Tm*B, 4D]
        QP = torch.zeros(Tm, B, A, dtype=dt, device=dev)
        AL = torch.zeros(Tm, B, S, dtype=torch.float32, device=dev)
        AWE = torch.zeros(Tm, B, De, dtype=dt, device=dev)
        GP = torch.zeros(Tm, B, De, dtype=dt, device=dev)    # f_beta pre-activation
        GT = torch.zeros(Tm, B, De, dtype=dt, device=dev)    # sigmoid gate
        XG = torch.zeros(Tm, B, De, dtype=dt, device=dev)    # gated context (LSTM input)
        ACT = torch.zeros(Tm, B, 4 * D, dtype=dt, device=dev)
        gates = torch.empty(B, 4 * D, dtype=dt, device=dev)
        we, be = m.att.weight.detach().view(-1), m.att.bias.detach()
        for t in range(Tm):
            bt = bts[t]
            h = Hs[t][:bt]
            ops.linear(h, W(m.dec_att.weight, dt), m.dec_att.bias.detach(), out=QP[t][:bt])
            ops.additive_attn_fwd(ATT_RELU, QP[t][:bt], kp[:bt], enc[:bt], we, be, 1.0, AWE[t][:bt], AL[t][:bt])
            ops.linear(h, W(m.f_beta.weight, dt), m.f_beta.bias.detach(), act=ACT_SIGMOID, preact=GP[t][:bt],
                       out=GT[t][:bt])
            ops.ew_mul(GT[t][:bt], AWE[t][:bt], XG[t][:bt])
            g = gates[:bt]
            ops.gemm(XG[t][:bt], True, w_ih[:, E:], True, bt, 4 * D, De, g, lda=De, ldb=E + De, ldc=4 * D,
                     residual=pre[t * B:t * B + bt], ldr=4 * D)
            ops.gemm(h, True, W(cs.weight_hh, dt), True, bt, 4 * D, D, g, lda=D, ldb=D, ldc=4 * D, beta=1.0,
                     bias=cs.bias_hh.detach())
            ops.lstm_cell_fwd(g, Cs[t][:bt], Cs[t + 1][:bt], Hs[t + 1][:bt], ACT[t][:bt])
        # predictions = fc(dropout(h)) for every step at once, b-major rows [B, Tm+1] (slot Tm
        # unused) so the shifted-CE kernel reads them in place
        Hb = torch.zeros(B, Tm + 1, D, dtype=dt, device=dev)
        idxT = torch.arange(Tm, dtype=torch.int32, device=dev)
        ops.gather_rows(Hs, idxT, Hb, B, Tm, D, B * D, D, D, (Tm + 1) * D, x_off=B * D)
        drop = (m.dropout.p, next_seed()) if (m.training and m.dropout.p > 0) else ops.NO_DROP
        Hd = ops.dropout_apply(Hb.view(B * (Tm + 1), D), drop) if drop[0] > 0 else Hb.view(B * (Tm + 1), D)
        logits = ops.linear(Hd, _pad_w(m.fc, dt), m.fc.bias._capk_pad_master)
        lens = torch.tensor(eff, dtype=torch.int32, device=dev)
        ops.mask_rows_by_length(logits.view(B, Tm + 1, Vp), lens)  # decoder.py:130-133: zeros elsewhere
        ctx.m, ctx.dims, ctx.bts = m, (B, S, De, A, D, E, V, Vp, Tm), bts
        ctx.saved = (enc, avg, kp, ids_t, emb, Hs, Cs, QP, AL, AWE, GP, GT, XG, ACT, Hd, drop, lens)
        ctx.logits = logits
        return logits.view(B, Tm + 1, Vp)[:, :Tm, :V], AL.permute(1, 0, 2)

    @staticmethod
    def backward(ctx, dpred, dalphas):
        m = ctx.m
        dt = m.cdtype
        B, S, De, A, D, E, V, Vp, Tm = ctx.dims
        bts = ctx.bts
        enc, avg, kp, ids_t, emb, Hs, Cs, QP, AL, AWE, GP, GT, XG, ACT, Hd, drop, lens = ctx.saved
        ctx.saved = None
        logits = ctx.logits
        ctx.logits = None
        dev = enc.device
        cs = m.decode_step
        # ---- output layer
        if dpred is None:
            dl = torch.zeros_like(logits)
        else:
            base = dpred._base
            if (base is not None and base.dim() == 2 and tuple(base.shape) == (B * (Tm + 1), Vp)
                    and base.data_ptr() == dpred.data_ptr() and base.is_contiguous()):
                dl = base
            else:
                dl = torch.zeros_like(logits)
                dl.view(B, Tm + 1, Vp)[:, :Tm, :V].copy_(dpred)
        ops.mask_rows_by_length(dl.view(B, Tm + 1, Vp), lens)
        ops.linear_dw(dl, Hd, m.fc.weight._capk_pad_grad)
        ops.colsum(dl, m.fc.bias._capk_pad_grad)
        dHb = ops.linear_dx(dl, _pad_w(m.fc, dt))  # [B*(Tm+1), D]
        if drop[0] > 0:
            dHb = ops.dropout_apply(dHb, drop)
        dHt = torch.empty(Tm, B, D, dtype=dt, device=dev)
        idxB = torch.arange(B, dtype=torch.int32, device=dev)
        ops.gather_rows(dHb, idxB, dHt, Tm, B, D, (Tm + 1) * D, D, D, B * D)
        # ---- gradient on the returned attention weights (the coverage regulariser)
        dw_const, dW_t = None, None
        if dalphas is not None:
            if dalphas.stride(1) == 0 and dalphas.dtype == torch.float32 and dalphas[:, 0].is_contiguous():
                dw_const = dalphas[:, 0]  # same [B, S] gradient for every step (expanded view)
            else:
                dW_t = dalphas.permute(1, 0, 2).float().contiguous()
        # ---- reverse-time recurrence.  dh = gradient w.r.t. h_{t+1} (= Hs[t+1]): the output
        # layer's dHt[t] plus, for rows still active at step t+1, the recurrent part.
        dh = torch.zeros(B, D, dtype=dt, device=dev)
        ops.copy_rows(dHt[Tm - 1], dh)
        dc = torch.zeros(B, D, dtype=torch.float32, device=dev)
        dG = torch.zeros(Tm, B, 4 * D, dtype=dt, device=dev)
        dQP = torch.zeros(Tm, B, A, dtype=dt, device=dev)
        dGP = torch.zeros(Tm, B, De, dtype=dt, device=dev)
        dEmb = torch.zeros(Tm, B, E, dtype=dt, device=dev)
        dkp = torch.zeros(B, S, A, dtype=torch.float32, device=dev)
        need_denc = ctx.needs_input_grad[0]
        dv = torch.zeros(B, S, De, dtype=torch.float32, device=dev) if need_denc else None
        dwe = torch.zeros(B, A, dtype=torch.float32, device=dev)
        dbe = torch.zeros(B, dtype=torch.float32, device=dev)
        dXG = torch.empty(B, De, dtype=dt, device=dev)
        tmp = torch.empty(B, De, dtype=dt, device=dev)
        dAWE = torch.empty(B, De, dtype=dt, device=dev)
        w_ih = W(cs.weight_ih, dt)
        we = m.att.weight.detach().view(-1)
        for t in range(Tm - 1, -1, -1):
            bt = bts[t]
            g = dG[t][:bt]
            ops.lstm_cell_bwd(ACT[t][:bt], Cs[t][:bt], dh[:bt], dc[:bt], g)
            ops.gemm(g, True, w_ih[:, E:], False, bt, De, 4 * D, dXG[:bt], lda=4 * D, ldb=E + De, ldc=De)
            ops.gemm(g, True, w_ih[:, :E], False, bt, E, 4 * D, dEmb[t][:bt], lda=4 * D, ldb=E + De, ldc=E)
            # gated context: XG = sigmoid(GP) * AWE
            ops.ew_mul(dXG[:bt], AWE[t][:bt], tmp[:bt])
            ops.act_bwd(tmp[:bt], GP[t][:bt], ACT_SIGMOID, out=dGP[t][:bt])
            ops.ew_mul(dXG[:bt], GT[t][:bt], dAWE[:bt])
            dw = None
            if dw_const is not None:
                dw = dw_const[:bt]
            elif dW_t is not None:
                dw = dW_t[t][:bt]
            ops.additive_attn_bwd(ATT_RELU, QP[t][:bt], kp[:bt], enc[:bt], we, 1.0, AL[t][:bt], dAWE[:bt],
                                  dQP[t][:bt], dkp, dv, dwe, dbe, dw_in=dw)
            # d h_t = dG W_hh + dQP W_dec + dGP W_fbeta (+ the output layer's dHt[t-1])
            res = dHt[t - 1][:bt] if t > 0 else None
            ops.gemm(g, True, W(cs.weight_hh, dt), False, bt, D, 4 * D, dh[:bt], lda=4 * D, ldb=D, ldc=D,
                     residual=res, ldr=D if res is not None else 0)
            ops.linear_dx(dQP[t][:bt], W(m.dec_att.weight, dt), out=dh[:bt], beta=1.0)
            ops.linear_dx(dGP[t][:bt], W(m.f_beta.weight, dt), out=dh[:bt], beta=1.0)
            if t > 0 and bts[t - 1] > bt:  # rows active at step t-1 only: output-layer gradient alone
                ops.copy_rows(dHt[t - 1][bt:bts[t - 1]], dh[bt:bts[t - 1]])
        # ---- batched weight gradients over all steps (inactive rows are zero)
        TB = Tm * B
        Hin = Hs[:Tm].reshape(TB, D)
        gG = dG.view(TB, 4 * D)
        ops.linear_dw(gG, Hin, G(cs.weight_hh))
        ops.colsum(gG, G(cs.bias_hh))
        ops.colsum(gG, G(cs.bias_ih))
        gw = G(cs.weight_ih)
        ops.gemm(gG, False, emb, False, 4 * D, E, TB, gw, lda=4 * D, ldb=E, ldc=E + De)
        ops.gemm(gG, False, XG.view(TB, De), False, 4 * D, De, TB, gw[:, E:], lda=4 * D, ldb=De, ldc=E + De)
        gq = dQP.view(TB, A)
        ops.linear_dw(gq, Hin, G(m.dec_att.weight))
        ops.colsum(gq, G(m.dec_att.bias))
        gp = dGP.view(TB, De)
        ops.linear_dw(gp, Hin, G(m.f_beta.weight))
        ops.colsum(gp, G(m.f_beta.bias))
        ops.colsum(dwe, G(m.att.weight).view(-1))
        ops.add_rows(dbe, G(m.att.bias), 1, 1, 1, 0, 0, B, 1, 0, 0, False)
        dkp2 = dkp.view(B * S, A)
        if dt != torch.float32:
            t_ = torch.empty(B * S, A, dtype=dt, device=dev)
            ops.cast(dkp2, t_)
            dkp2 = t_
        enc2 = enc.view(B * S, De)
        ops.linear_dw(dkp2, enc2, G(m.enc_att.weight))
        ops.colsum(dkp2, G(m.enc_att.bias))
        ops.zero_(G(m.embedding.weight))
        ops.embedding_bwd(ids_t, dEmb.view(TB, E), -1, G(m.embedding.weight), None, 0)
        # ---- initial state -> h_lin / c_lin (-> mean pixel)
        dc_t = dc if dt == torch.float32 else ops.cast(dc, torch.empty(B, D, dtype=dt, device=dev))
        ops.linear_dw(dh, avg, G(m.h_lin.weight))
        ops.colsum(dh, G(m.h_lin.bias))
        ops.linear_dw(dc_t, avg, G(m.c_lin.weight))
        ops.colsum(dc_t, G(m.c_lin.bias))
        denc = None
        if need_denc:
            davg = ops.linear_dx(dh, W(m.h_lin.weight, dt))
            ops.linear_dx(dc_t, W(m.c_lin.weight, dt), out=davg, beta=1.0)
            dv2 = dv.view(B * S, De)
            denc = torch.empty(B * S, De, dtype=dt, device=dev)
            ops.cast(dv2, denc)
            ops.linear_dx(dkp2, W(m.enc_att.weight, dt), out=denc, beta=1.0)
            ops.avgpool_bwd(davg, B, S, 1, De, 1, 1, dx=denc, beta=1.0)
            denc = denc.view(B, S, De)
        return denc, None, None, None, None


# ------------------------------------------------------------------- loss ----
class _LegacyLossFn(torch.autograd.Function):
    """train.py:92-101: CE over pack_padded_sequence(scores / targets, decode_lengths)
    (= mean over the active (b, t)) + ((1 - alphas.sum(dim=1)) ** 2).mean()."""

    @staticmethod
    def forward(ctx, predictions, alphas, captions, dec_len):
        B, Tm, V = predictions.shape
        ld = predictions.stride(1)
        if predictions.stride(2) == 1 and ld % 8 == 0 and predictions.stride(0) == (Tm + 1) * ld:
            base = predictions.as_strided((B * (Tm + 1), ld), (ld, 1))
        else:
            ld = _pad64(V)
            base = torch.zeros(B * (Tm + 1), ld, dtype=predictions.dtype, device=predictions.device)
            base.view(B, Tm + 1, ld)[:, :Tm, :V].copy_(predictions)
        dev = predictions.device
        # targets[b, j] = caption token j for j < dec_len[b] + 1, else ignored (-100)
        lens = torch.tensor([d + 1 for d in dec_len], device=dev).view(B, 1)
        pos = torch.arange(Tm + 1, device=dev).view(1, Tm + 1)
        tg = torch.where(pos < lens, captions[:, :Tm + 1], torch.full_like(captions[:, :Tm + 1], -100)).contiguous()
        loss = ops.shifted_ce(base, tg, B, Tm + 1, V, -100, want_loss=True)
        al = alphas.permute(1, 0, 2)
        if not al.is_contiguous() or al.dtype != torch.float32:
            al = al.float().contiguous()
        ops.attn_coverage_reg(al, loss_acc=loss[:1])
        ctx.base, ctx.tg, ctx.al = base, tg, al
        ctx.dims = (B, Tm, V)
        return loss[0]

    @staticmethod
    def backward(ctx, dloss):
        B, Tm, V = ctx.dims
        base, tg, al = ctx.base, ctx.tg, ctx.al
        ctx.base = ctx.tg = ctx.al = None
        gs = dloss.reshape(1).float().contiguous()
        dbase = torch.empty_like(base)
        ops.shifted_ce(base, tg, B, Tm + 1, V, -100, want_loss=False, dlogits=dbase, grad_scale=gs)
        ld = base.shape[1]
        coef = torch.empty(B, al.shape[2], dtype=torch.float32, device=base.device)
        ops.attn_coverage_reg(al, grad_scale=gs, coef=coef)
        dpred = dbase.view(B, Tm + 1, ld)[:, :Tm, :V]
        dal = coef.view(B, 1, -1).expand(B, Tm, coef.shape[1])
        return dpred, dal, None, None


class LegacyCaptionLoss(nn.Module):
    """criterion = nn.CrossEntropyLoss() on the packed scores + the attention regulariser
    (train.py:92-101; D12: the reference never defines `criterion`, CE is its evident intent)."""

    def forward(self, predictions, alphas, captions, dec_len):
        if any(dec_len[i] < dec_len[i + 1] for i in range(len(dec_len) - 1)):
            raise RuntimeError("`lengths` array must be sorted in decreasing order (pack_padded_sequence)")
        return _LegacyLossFn.apply(predictions, alphas, captions, tuple(int(d) for d in dec_len))


# -------------------------------------------------------------- optimizer ----
class LegacyAdam:
    """torch.optim.Adam(decoder.parameters(), lr=4e-4) with the per-element gradient clamp
    of train.py:105-110 (clamp_(-grad_clip, grad_clip) before every step); fused: one
    clamp pass + one Adam (AdamW kernel with weight decay 0 == Adam) pass per group."""

    def __init__(self, store, lr=4e-4, betas=(0.9, 0.999), eps=1e-8, grad_clip=5.0):
        self.store = store
        self.param_groups = [{"lr": lr}]
        self.betas, self.eps, self.grad_clip = betas, eps, grad_clip
        self.m = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.v = {g: torch.zeros_like(store.master[g]) for g in store.groups}
        self.n = 0

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    def step(self):
        self.n += 1
        st = self.store
        for g in st.groups:
            n = st.required_numel[g]
            if n == 0:
                continue
            if self.grad_clip is not None:
                ops.clamp_(st.grad[g][:n], -self.grad_clip, self.grad_clip)
            sh = None if st.bf16[g] is None else st.bf16[g][:n]
            ops.adamw(st.master[g][:n], st.grad[g][:n], self.m[g][:n], self.v[g][:n], sh, self.lr, 0.0,
                      self.betas[0], self.betas[1], self.eps, self.n)

    def zero_grad(self):
        self.store.relink_grads()


def train_step(encoder, decoder, optimizer, criterion, imgs, caps, caplens):
    """One batch of train.py:train() (lines 84-112): encoder forward (train-mode BN), decoder,
    packed CE + attention regulariser, backward, clamp + Adam.  The reference also back-
    propagates into the encoder, whose gradients no optimizer consumes; here the encoder
    output is detached, so the observable state (decoder weights, BN buffers) is identical."""
    with torch.no_grad():
        feats = encoder(imgs)
    scores, caps_sorted, decode_lengths, alphas = decoder(feats, caps, caplens)
    loss = criterion(scores, alphas, caps_sorted, decode_lengths)
    optimizer.zero_grad()
    loss.backward()
    optimizer.step()
    return loss


def decay_lr(optimizer, batch_index, every=1000, factor=0.8):
    """train.py:116-123: lr *= 0.8 every 1000 batches (i % 1000 == 0 and i != 0)."""
    if batch_index % every == 0 and batch_index != 0:
        for g in optimizer.param_groups:
            g["lr"] = g["lr"] * factor
