"""Markdown table of a strict-parity record (tests/test_gpu_parity_strict.py
writes gpurun_out/parity_strict.json): per case and frame, bits of the product
and the oracle, differing symbols / indexes, the first flip and its tie
distance, and the replay (the oracle re-run with the product's symbols forced
at its tie positions: its bits must equal the product's).

    python scripts/parity_table.py profiles/r04f_parity_strict.json
"""
import json
import sys


def main(path):
    d = json.load(open(path))
    print("| case | frame | bits (product / oracle) | Δsym / Δidx of all | first flip (tie distance) | replay: bits, Δsym / Δidx | max tie distance | ΔPSNR dB |")
    print("|---|---|---|---|---|---|---|---|")
    for case, frames in d.items():
        for i, fr in enumerate(frames):
            ff = fr.get("first_flip")
            ffs = f"{ff['kind']} call {ff['call']} ({max(ff['tie_dist']):.1e})" if ff else "—"
            rp = fr.get("replay")
            rps = (f"{rp['bits_replay']} ({'=' if rp['bits_replay'] == fr.get('bits') else '≠'}), "
                   f"{rp['sym_diff']} / {rp['idx_diff']}") if rp else "—"
            bits = f"{fr.get('bits')} / {fr.get('bits_oracle')}"
            dp = abs(fr.get("psnr", 0) - fr.get("psnr_oracle", 0)) if "psnr" in fr else float("nan")
            print(f"| {case} | {fr.get('t', i)} | {bits} | {fr['sym_diff']} / {fr['idx_diff']} of {fr['symbols']} | {ffs} | "
                  f"{rps} | {fr.get('max_tie_dist', 0):.1e} | {dp:.1e} |")


if __name__ == "__main__":
    main(sys.argv[1])
