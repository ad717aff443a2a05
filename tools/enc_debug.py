"""Compare the product text encoder with the oracle restatement stage by stage on the GPU (eval, fp32)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "matcha-tts-etu-upmc-ensam_amd"), str(ROOT)]
import torch
from oracle import matcha_oracle as MO
from matcha.models.matcha_tts import MatchaTTS
from matcha.utils.model import sequence_mask
from matcha.models.components import _ops as O

dev = torch.device("cuda")
torch.manual_seed(0)
model = MatchaTTS(n_vocab=150, out_channels=80, hidden_channels=192).to(dev).eval()
enc = model.encoder
ora = MO.TextEncoderO(150).to(dev).eval()
for p in enc.parameters():
    p.data.normal_(0, 0.05)
missing = ora.load_state_dict(enc.state_dict(), strict=False)
print("load:", missing)
B, T = 3, 23
x = torch.randint(1, 150, (B, T), device=dev)
lens = torch.tensor([23, 17, 11], device=dev)
m = sequence_mask(lens, T).float()
mv = m.bool()
def cmp(name, a_tm, b_cm):
    a = a_tm[mv]; b = b_cm.transpose(1, 2)[mv]
    print(f"{name:28s} max|d| {((a - b).abs().max()).item():.3e}  max|ref| {b.abs().max().item():.3e}")
with torch.no_grad():
    e = enc.embedding(x) * (192 ** 0.5)
    pa = enc.prenet.forward_tm(e, m)
    pb = ora.prenet(e.transpose(1, 2), m.unsqueeze(1))
    cmp("prenet", pa, pb)
    # prenet stage 1: conv + LN/relu
    h1 = O.conv_tm(e, enc.prenet.convolutions[0].weight, enc.prenet.convolutions[0].bias, mask=m)
    c = ora.prenet.convolutions[0](e.transpose(1, 2) * m.unsqueeze(1))
    cmp("prenet conv0 (k5)", h1, c)
    ln = enc.prenet.normalizations[0]
    h2 = O.layer_norm_tm(h1, ln.weight, ln.bias, ln.eps, relu=True)
    c2 = torch.relu(ln(c.transpose(1, 2))).transpose(1, 2)
    cmp("prenet LN+relu", h2, c2)
    # one encoder layer
    h = pb.transpose(1, 2).contiguous()
    L = enc.encoder
    amask = m.unsqueeze(1).unsqueeze(2) * m.unsqueeze(1).unsqueeze(-1)
    att = L.attention_layers[0]
    o = att.attend_tm(h, m, (m - 1) * 1e4)
    ob = ora.encoder.attention_layers[0]
    # oracle attention output before output_conv
    xc = h.transpose(1, 2) * m.unsqueeze(1)
    Bq, C, Tq = xc.shape
    q = ob.query_conv(xc).view(Bq, 2, 96, Tq).transpose(2, 3)
    k = ob.key_conv(xc).view(Bq, 2, 96, Tq).transpose(2, 3)
    v = ob.value_conv(xc).view(Bq, 2, 96, Tq).transpose(2, 3)
    q2, k2 = MO.rope(q.cpu(), 48).to(dev), MO.rope(k.cpu(), 48).to(dev)
    s = (q2 @ k2.transpose(-1, -2)) / 96 ** 0.5
    s = s.masked_fill(amask == 0, -1e4)
    oo = (torch.softmax(s, -1) @ v).transpose(2, 3).contiguous().view(Bq, C, Tq)
    cmp("attention (pre out-conv)", o, oo)
    qkv = O.linear_tm(h, (att.query_conv.weight, att.key_conv.weight, att.value_conv.weight),
                      torch.cat([att.query_conv.bias, att.key_conv.bias, att.value_conv.bias]), in_scale=m)
    cmp("q projection", qkv[..., :192], q.transpose(2, 3).reshape(Bq, C, Tq))
    cos, sin = att.query_rope.tables(Tq, dev)
    qr = O.rope_tm(qkv, cos, sin, 2, 48)
    cmp("q rope", qr[..., :192], q2.transpose(2, 3).reshape(Bq, C, Tq))
    cmp("k rope", qr[..., 192:384], k2.transpose(2, 3).reshape(Bq, C, Tq))
    ea = L.forward_tm(h, m)
    ora_c = MO.TextEncoderO(150).eval()
    ora_c.load_state_dict(enc.state_dict(), strict=False)
    eb = ora_c.encoder(pb.cpu(), m.unsqueeze(1).cpu()).to(dev)
    cmp("encoder (6 layers)", ea, eb)
    mu, logw, _ = enc(x, lens)
    mub, logwb, _ = [t.to(dev) for t in ora_c(x.cpu(), lens.cpu())]
    cmp("mu", mu.transpose(1, 2), mub)
    cmp("logw", logw.transpose(1, 2), logwb)
    dpa = enc.duration_predictor.forward_tm(eb.transpose(1, 2).contiguous(), m)
    cmp("duration predictor (same in)", dpa, ora.duration_predictor(eb, m.unsqueeze(1)))
    # first encoder layer, piecewise
    xo = h.transpose(1, 2) * m.unsqueeze(1)
    x1b = ora_c.encoder.norm_layers_1[0]((xo + ora_c.encoder.attention_layers[0](xo.cpu(), amask.cpu()).to(dev)).transpose(1, 2).cpu()).to(dev)
    x1a = O.layer_norm_tm(O.linear_tm(o, att.output_conv.weight, att.output_conv.bias, residual=h), L.norm_layers_1[0].weight, L.norm_layers_1[0].bias)
    cmp("layer0 LN1", x1a, x1b.transpose(1, 2))
    # layer-by-layer
    ha = h.clone()
    hb = h.transpose(1, 2).cpu()
    mc = m.unsqueeze(1).cpu()
    amc = amask.cpu()
    E = ora_c.encoder
    for i in range(6):
        att = L.attention_layers[i]
        o = att.attend_tm(ha, m, (m - 1) * 1e4)
        xa = O.layer_norm_tm(O.linear_tm(o, att.output_conv.weight, att.output_conv.bias, residual=ha),
                             L.norm_layers_1[i].weight, L.norm_layers_1[i].bias)
        ffa = L.ffn_layers[i].forward_tm(xa, m, residual=xa)
        ha_new = O.layer_norm_tm(ffa, L.norm_layers_2[i].weight, L.norm_layers_2[i].bias)
        xb = hb * mc
        xb = E.norm_layers_1[i]((xb + E.attention_layers[i](xb, amc)).transpose(1, 2)).transpose(1, 2)
        cmp(f"L{i} LN1", xa, xb.to(dev))
        ffb = E.ffn_layers[i](xb, mc)
        cmp(f"L{i} ffn+res", ffa, (xb + ffb).to(dev))
        hb = E.norm_layers_2[i]((xb + ffb).transpose(1, 2)).transpose(1, 2)
        cmp(f"L{i} out", ha_new, hb.to(dev))
        ha = ha_new
