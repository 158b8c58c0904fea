#!/usr/bin/env python3
"""Write the distinct Convolution / InnerProduct ops of full nets (the executor's plan, no GPU)
as an op list in the reference's op-line dialect, for tools/tune.py --sets nets.

  python tools/net_ops.py --img 20 --out boda-1_amd/tuning/net-ops-b20.txt
"""
import argparse
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "boda-1_amd", "bin", "boda_hip_rtc_fwd")
NETS = ["alexnet_ng_conv", "nin_imagenet", "googlenet_conv", "resnet-50", "vgg_19"]


def op_line(B, IC, H, W, OC, KY, KX, sy, sx, py, px):
    OH, OW = (H + 2 * py - KY) // sy + 1, (W + 2 * px - KX) // sx + 1
    return ("(str_vals=(type=Convolution),nda_vals=(biases=(dims=(out_chan=%d)),filts=(dims=(out_chan=%d,in_chan=%d,"
            "y=%d,x=%d)),in=(dims=(img=%d,chan=%d,y=%d,x=%d)),in_pad=(tn=none,dims=(y=%d,x=%d)),kern_sz=(tn=none,"
            "dims=(y=%d,x=%d)),out=(dims=(img=%d,chan=%d,y=%d,x=%d)),out_chans=(tn=uint32_t,v=%d),stride=(tn=none,"
            "dims=(y=%d,x=%d))))" % (OC, OC, IC, KY, KX, B, IC, H, W, py, px, KY, KX, B, OC, OH, OW, OC, sy, sx))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=20)
    ap.add_argument("--out", default=os.path.join(ROOT, "boda-1_amd", "tuning", "net-ops-b20.txt"))
    a = ap.parse_args()
    lines = []
    for net in NETS:
        pt = os.path.join(ROOT, "tests", "golden", "nets", net + ".prototxt")
        plan = json.loads(subprocess.run([BIN, "--net", pt, "--img", str(a.img), "--plan-json"], check=True,
                                         capture_output=True, text=True).stdout)
        dims = {i["name"]: i["dims"] for i in plan["inputs"]}
        for o in plan["ops"]:
            B, C, H, W = dims[o["bots"][0]]
            if o["type"] == "Convolution":
                d = (B, C, H, W, o["out_chans"], o["k"][0], o["k"][1], o["s"][0], o["s"][1], o["p"][0], o["p"][1])
            elif o["type"] == "InnerProduct":  # a conv whose kernel covers the input (ipconv)
                d = (B, C, H, W, o["out_chans"], H, W, 1, 1, 0, 0)
            else:
                d = None
            for t in o["tops"]:
                dims[t] = o["out_dims"]
            if d is not None:
                l = op_line(*d)
                if l not in lines:
                    lines.append(l)
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("wrote %d ops to %s" % (len(lines), a.out))


if __name__ == "__main__":
    main()
