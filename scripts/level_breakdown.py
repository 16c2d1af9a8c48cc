"""Per-hourglass-level time from op_profile.py's parse output (eager + separators, so small
launches are inflated by ~1 us each).  usage: python scripts/level_breakdown.py ops.txt"""
import collections
import re
import sys

LV = {131072: "64", 32768: "32", 8192: "16", 2048: "8", 512: "4", 524288: "128"}


def m_of(fn, a):
    if fn == "hgk_conv_fwd":
        return a[4] * a[5] * a[6]
    if fn == "hgk_conv_fwd_bnbwd":
        return a[2] * a[3] * a[4]
    if fn in ("hgk_bn_finalize", "hgk_bn_bwd_finalize"):
        return a[1]
    if fn == "hgk_bn_bwd_finalize_apply":
        return a[2]
    if fn in ("hgk_bn_bwd_apply", "hgk_bn_stats", "hgk_bn_bwd_reduce"):
        return a[1]
    if fn == "hgk_conv_wgrad_accum":
        return a[5] * a[6] * a[7]
    return None


def main():
    lv = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    byop = collections.defaultdict(float)
    for ln in open(sys.argv[1]):
        m = re.match(r"\s*([\d.]+) us n=\s*(\d+) avg=\s*([\d.]+)\s+(\S+)\s*(.*)", ln)
        if not m:
            continue
        t, n, fn = float(m[1]), int(m[2]), m[4]
        a = [int(x) for x in m[5].split() if re.fullmatch(r"-?\d+", x)]
        key = LV.get(m_of(fn, a), "other")
        lv[key] += t
        cnt[key] += n
        byop[(key, fn)] += t
    tot = sum(lv.values())
    print(f"total {tot:.0f} us")
    for k in sorted(lv, key=lambda k: -lv[k]):
        print(f"level {k:>5}: {lv[k]:8.0f} us  {cnt[k]:5d} launches  {lv[k] / tot:.3f}")
        for (kk, fn), t in sorted(byop.items(), key=lambda kv: -kv[1]):
            if kk == k and t > 0.02 * lv[k]:
                print(f"      {fn:28s} {t:8.0f}")


if __name__ == "__main__":
    main()
