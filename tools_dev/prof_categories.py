"""Group a rocprofv3 kernel-stats CSV into categories (ms per step).
  python tools_dev/prof_categories.py <run_kernel_stats.csv> <steps_in_trace>"""
import csv
import re
import sys

CATS = [
    ("hipBLASLt/rocBLAS GEMM", r"^(Custom_)?Cijk_"),
    ("attention (aotriton)", r"attn_fwd|bwd_kernel_d|bwd_preprocess"),
    ("MIOpen conv", r"miopen|Im2d2Col|Col2Im|igemm|ConvHip|conv_|gridwise|naive_conv|Sp3Asm|xdlops"),
    ("own HIP kernels", r"dwr_|dw_fwd|dw_bwd|gn_fwd|gn_bwd|gelu_fwd|gelu_bwd|lsr_|blur_|updn|bias_act|flrelu|codebook"),
    ("torch reduce", r"reduce_kernel"),
    ("torch layer/group norm", r"layer_norm|group_norm|GroupNorm|LayerNorm"),
    ("torch copy/cast", r"copy_kernel|direct_copy|copyBuffer|bfloat16_copy|float32_copy|cat_|CatArray"),
    ("torch elementwise", r"elementwise|Functor|vectorized"),
    ("optimizer", r"multi_tensor|adam|Adam|foreach"),
]


def main():
    path, steps = sys.argv[1], float(sys.argv[2])
    tot = {}
    other = {}
    for r in csv.DictReader(open(path)):
        n, t = r["Name"], float(r["TotalDurationNs"])
        for cat, pat in CATS:
            if re.search(pat, n):
                tot[cat] = tot.get(cat, 0) + t
                break
        else:
            tot["other"] = tot.get("other", 0) + t
            other[n[:90]] = other.get(n[:90], 0) + t
    s = sum(tot.values())
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{v / steps / 1e6:9.2f} ms/step  {100 * v / s:5.1f} %  {k}")
    print("top 'other':")
    for k, v in sorted(other.items(), key=lambda kv: -kv[1])[:12]:
        print(f"{v / steps / 1e6:9.2f} ms/step  {k}")


if __name__ == "__main__":
    main()
