import sys, torch
sys.path.insert(0, "/root/repo")
from dcvc_amd import hip as K
torch.manual_seed(0)
dev = torch.device("cuda", 0)
for (cin, cout, H, W) in ((384, 1024, 68, 120), (192, 768, 68, 120)):
    w1 = torch.randn(cout, cin, 1, 1) / cin ** 0.5
    b1 = torch.randn(cout) * 0.1
    c1 = K.ConvW(w1, b1, 1, K.BF16, dev)
    x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.F32)
    hf = K.conv(c1, x, out_dtype=K.F32, act=K.ACT_LRELU, slope=0.1)
    hb = K.conv(c1, x, out_dtype=K.BF16, act=K.ACT_LRELU, slope=0.1)
    print(K.lib().dcvc_last_kernel().decode())
    ref = hf.t().to(torch.bfloat16)
    d = (ref.view(torch.int16) != hb.t().view(torch.int16))
    print(cin, cout, "h mismatches:", int(d.sum()), "of", d.numel())
    if d.any():
        i = d.nonzero()[0]
        print(" example", hf.t()[tuple(i)].item(), ref[tuple(i)].item(), hb.t()[tuple(i)].item())
    w2 = torch.randn(cin, cout, 1, 1) / cout ** 0.5
    c2 = K.ConvW(w2, torch.randn(cin) * 0.1, 1, K.BF16, dev)
    of = K.conv(c2, hf, out_dtype=K.F32, act=K.ACT_LRELU, slope=0.1, res=x)
    kf = K.lib().dcvc_last_kernel().decode()
    ob = K.conv(c2, hb, out_dtype=K.F32, act=K.ACT_LRELU, slope=0.1, res=x)
    kb = K.lib().dcvc_last_kernel().decode()
    print(" ffn2 kernels", kf, "|", kb, "out mismatches:", int((of.t() != ob.t()).sum()))
