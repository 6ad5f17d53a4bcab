"""Extract the reference's published sub-block GPU decoder BER/FER (the P sweep) into a fixture.

Source: /root/reference/ITTC/CUDA/FinalResult/{8,12,16,24,32}_4Blocks_Bian_Max_10000Fs_Iter25_*.txt,
the stdout of turboDecoderBianJieZhi.cu (main: :600-700) with BLOCK_NUM = 8..32, i.e. P = 4 *
BLOCK_NUM sub-blocks of 6144/P steps; 10000 frames per Eb/N0 point (FRAME_NUM), Eb/N0 0..1 dB in
0.1 steps, 25 iterations, "Ber=%f" / "Fer=%f" per iteration (6 decimals).  The FinalBer/Iters*_P
tables are columns of these files (FinalResult/ber.sh).  Data only; writes
tests/golden/psweep_published.json.
"""
import glob
import json
import os
import re

SRC = "/root/reference/ITTC/CUDA/FinalResult"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "psweep_published.json")


def parse(path):
    pts, cur = [], None
    for line in open(path, errors="replace"):
        m = re.match(r"Eb/No=([0-9.]+)dB", line.strip())
        if m:
            cur = {"ebn0_db": float(m.group(1)), "ber": [], "fer": []}
            pts.append(cur)
            continue
        m = re.match(r"---Ber=([0-9.eE+-]+)", line.strip())
        if m:
            cur["ber"].append(float(m.group(1)))
        m = re.match(r"---Fer=([0-9.eE+-]+)", line.strip())
        if m:
            cur["fer"].append(float(m.group(1)))
        m = re.match(r"throughput: ([0-9.eE+-]+)Mbps", line.strip())
        if m:
            cur["throughput_mbps"] = float(m.group(1))
    return pts


def main():
    res = {"source": "ITTC/CUDA/FinalResult/*_4Blocks_Bian_Max_10000Fs_Iter25_*.txt",
           "decoder": "turboDecoderBianJieZhi.cu: Max-Log-MAP fp32, P sub-blocks, NII, concurrent SISOs, Le x0.77",
           "K": 6144, "frames_per_point": 10000, "iterations": 25, "P": {}}
    for f in sorted(glob.glob(os.path.join(SRC, "*_4Blocks_Bian_Max_10000Fs_Iter25_*.txt"))):
        P = 4 * int(os.path.basename(f).split("_")[0])
        pts = parse(f)
        assert len(pts) == 11 and all(len(p["ber"]) == 25 and len(p["fer"]) == 25 for p in pts), f
        res["P"][str(P)] = pts
    with open(OUT, "w") as fp:
        json.dump(res, fp, indent=0)
    print(OUT, sorted(res["P"], key=int))


if __name__ == "__main__":
    main()
