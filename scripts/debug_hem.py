import sys, torch, numpy as np
sys.path.insert(0, '.')
from tests.hem_fixtures import HEMGolden
from oracle import hem_oracle as O
from oracle import rans_oracle as R
from dcvc_amd.hem import IntraNoAR
from dcvc_amd.layers import Precision
from dcvc_amd import hip as K
g = HEMGolden()
x, xp = g.frame_tensor("A", 0)
qi = g.q("A")[0]
orc = O.IntraOracle(g.i_state_dict(), R.pmf_to_quantized_cdf)
P = orc.P
net = IntraNoAR(precision=Precision.parity()).load_state_dict(g.i_state_dict())
net.update(force=True)
q = round(qi * 100) / 100
def cmp(name, a, b):
    a = a.float().cpu(); b = b.float().cpu()
    print(f"{name:12s} maxabs {float((a-b).abs().max()):.3e}  ref maxabs {float(b.abs().max()):.3e}")
with torch.no_grad():
    qo = O.lower_bound_q(P, "q_basic", q)
    yo_raw = O.enc_model(P, "enc", xp)
    yo = yo_raw / qo
    zo = torch.round(O.hyper_enc(P, "hyper_enc", yo))
    qs_o, sc_o, me_o = orc._prior(zo)
    xa = K.from_nchw(xp.cuda(), K.F32)
    qg = net._q(q)
    yg_raw = net.enc(xa)
    cmp("enc", yg_raw.nchw(), yo_raw)
    yg = K.channel_div(yg_raw, qg)
    cmp("y", yg.nchw(), yo)
    zg = net.henc(yg)
    cmp("z_hat", zg.nchw(), zo)
    # feed the oracle's z to isolate the prior path
    zt = K.from_nchw(zo.cuda(), K.F32)
    buf = net._params(zt)
    t = buf.nchw()
    N = net.N
    cmp("means", t[:, N:2*N], me_o)
    cmp("scales", t[:, 2*N:3*N], sc_o)
    cmp("qstep", t[:, 3*N:4*N], qs_o)
    # first blocks of the encoder
    h = net.enc.blocks[0](xa)
    ho = O.residual_block_with_stride(P, "enc.0", xp)
    cmp("enc.0", h.nchw(), ho)
    h2 = net.enc.blocks[1](h)
    ho2 = O.residual_block(P, "enc.1", ho)
    cmp("enc.1", h2.nchw(), ho2)
    # full dual prior on identical inputs: the oracle's y, params
    yt = K.from_nchw(yo.cuda(), K.F32)
    buf = net._params(zt)
    sbsym = [torch.empty(N // 2 * yt.H * yt.W, dtype=torch.int32, device="cuda") for _ in range(2)]
    sbidx = [torch.empty(N // 2 * yt.H * yt.W, dtype=torch.int16, device="cuda") for _ in range(2)]
    yhat = net.prior.encode(yt, buf, qg, sbsym, sbidx, net.scale_table)
    q0, q1, s0, s1, yh_o = O.dual_prior(P, yo, me_o, sc_o, qs_o, lambda t: O.seq3(P, "y_spatial_prior", t), write=True)
    for k, (qq, ss) in enumerate(((q0, s0), (q1, s1))):
        gs = sbsym[k].cpu().numpy()
        os_ = qq.reshape(-1).int().numpy()
        gi = sbidx[k].cpu().numpy()
        oi = O.build_indexes(ss, orc.tab_y[3], orc.tab_y[4]).reshape(-1).numpy()
        d = np.nonzero(gs != os_)[0]
        print(f"step {k}: sym diff {d.size} idx diff {(gi != oi).sum()} of {gs.size}")
        if d.size:
            j = d[:5]
            print("   gpu", gs[j], "orc", os_[j])
    cmp("y_hat", yhat.nchw() * 1.0, yh_o * qo.view(1, -1, 1, 1))
    # spatial prior output on the same buffer
    smg = net.prior.spatial(buf)
    h00 = yh_o  # unused
