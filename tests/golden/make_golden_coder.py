"""Known-answer vectors for pmf_to_quantized_cdf, produced by the REFERENCE's
own ops.cpp (DCVC-DC/src/cpp/ops/ops.cpp:24-82) compiled into oracle/_ref by
`make ref`.  Run here only:  python tests/golden/make_golden_coder.py"""
import importlib.machinery
import importlib.util
import os
import sysconfig

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main():
    so = os.path.join(REPO, "oracle", "_ref", "MLCodec_CXX" + sysconfig.get_config_var("EXT_SUFFIX"))
    loader = importlib.machinery.ExtensionFileLoader("MLCodec_CXX", so)
    spec = importlib.util.spec_from_file_location("MLCodec_CXX", so, loader=loader)
    ref = importlib.util.module_from_spec(spec)
    loader.exec_module(ref)
    g = np.random.Generator(np.random.PCG64(123))
    pmfs = []
    for n in (2, 3, 5, 17, 64, 101, 103):
        for kind in range(4):
            if kind == 0:      # dirichlet
                p = g.dirichlet(np.ones(n))
            elif kind == 1:    # peaked with many zero bins (forces stealing)
                p = np.zeros(n)
                p[n // 2] = 1.0 - 1e-6 * (n - 1)
                p[p == 0] = 1e-7
            elif kind == 2:    # laplace-like discretised, tiny tails
                x = np.arange(n) - n // 2
                p = np.exp(-np.abs(x) / max(1.0, n / 20))
                p /= p.sum()
            else:              # exact zeros and one negative rounding residue
                p = g.dirichlet(np.ones(n) * 0.2)
                p[::3] = 0.0
                p[-1] = -0.0
                if p.sum() == 0:   # all-zero pmf divides by zero in ops.cpp:41
                    p[n // 2] = 1.0
            pmfs.append(p.astype(np.float32))
    cdfs = [np.asarray(ref.pmf_to_quantized_cdf(p.tolist(), 16), dtype=np.uint32) for p in pmfs]
    out = {}
    for k, (p, c) in enumerate(zip(pmfs, cdfs)):
        out[f"pmf{k}"] = p
        out[f"cdf{k}"] = c
    np.savez_compressed(os.path.join(HERE, "coder_golden.npz"), **out)
    print(len(pmfs), "vectors")


if __name__ == "__main__":
    main()
