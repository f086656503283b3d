"""Oracle restatement of the legacy Show-Attend-Tell path.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Parameters are dicts keyed by the reference state-dict names of models/decoder.py
``Decoder`` (enc_att, dec_att, att, decode_step.{weight,bias}_{ih,hh}, h_lin, c_lin,
f_beta, fc, embedding).  Plain PyTorch-CPU fp32, following the reference line by line
except that enc_att(encoder_out) is evaluated once (it does not depend on t).
"""
import torch
import torch.nn.functional as F


def legacy_decoder(p, encoder_out, captions, lengths, dropout_p=0.0):
    """Decoder.forward (models/decoder.py:120-176): returns (predictions [B,T,V], alphas [B,T,S])."""
    B = encoder_out.shape[0]
    enc = encoder_out.reshape(B, -1, encoder_out.shape[-1])
    S = enc.shape[1]
    dec_len = [x - 1 for x in lengths]
    Tm = max(dec_len)
    V = p["fc.weight"].shape[0]
    emb = F.embedding(captions, p["embedding.weight"])                       # 135-136
    avg = enc.mean(dim=1)                                                     # 141-143
    h = F.linear(avg, p["h_lin.weight"], p["h_lin.bias"])
    c = F.linear(avg, p["c_lin.weight"], p["c_lin.bias"])
    preds = torch.zeros(B, Tm, V)
    alphas = torch.zeros(B, Tm, S)
    enc_att_all = F.linear(enc, p["enc_att.weight"], p["enc_att.bias"])       # 155 (hoisted)
    for t in range(Tm):
        bt = sum(1 for l in dec_len if l > t)                                 # 153
        dec_att = F.linear(h[:bt], p["dec_att.weight"], p["dec_att.bias"])    # 156
        att = F.linear(F.relu(enc_att_all[:bt] + dec_att.unsqueeze(1)), p["att.weight"], p["att.bias"]).squeeze(2)
        alpha = torch.softmax(att, dim=1)                                     # 159
        awe = (enc[:bt] * alpha.unsqueeze(2)).sum(dim=1)                      # 160-161
        gate = torch.sigmoid(F.linear(h[:bt], p["f_beta.weight"], p["f_beta.bias"]))  # 163
        awe = gate * awe
        x = torch.cat([emb[:bt, t], awe], dim=1)                              # 166-168
        gates = F.linear(x, p["decode_step.weight_ih"], p["decode_step.bias_ih"]) + \
            F.linear(h[:bt], p["decode_step.weight_hh"], p["decode_step.bias_hh"])  # nn.LSTMCell
        i, f, g, o = gates.chunk(4, 1)
        c = torch.sigmoid(f) * c[:bt] + torch.sigmoid(i) * torch.tanh(g)
        h = torch.sigmoid(o) * torch.tanh(c)
        hd = F.dropout(h, dropout_p, training=dropout_p > 0)
        preds[:bt, t] = F.linear(hd, p["fc.weight"], p["fc.bias"])            # 174-176
        alphas[:bt, t] = alpha
    return preds, alphas


def legacy_loss(preds, alphas, captions, lengths):
    """train.py:92-101: CE over the packed (b, t < dec_len[b]) scores + doubly stochastic term."""
    dec_len = [x - 1 for x in lengths]
    rows, tgts = [], []
    for b, d in enumerate(dec_len):
        rows.append(preds[b, :d])
        tgts.append(captions[b, 1:d + 1])
    ce = F.cross_entropy(torch.cat(rows), torch.cat(tgts))
    return ce + ((1. - alphas.sum(dim=1)) ** 2).mean()


def clamp_adam_step(params, grads, lr=4e-4, clip=5.0, betas=(0.9, 0.999), eps=1e-8):
    """train.py:105-112 first step: clamp grads to [-clip, clip], torch Adam step 1."""
    out = {}
    b1, b2 = betas
    for n, w in params.items():
        g = grads[n].clamp(-clip, clip)
        m = (1 - b1) * g
        v = (1 - b2) * g * g
        mh, vh = m / (1 - b1), v / (1 - b2)
        out[n] = w - lr * mh / (vh.sqrt() + eps)
    return out
