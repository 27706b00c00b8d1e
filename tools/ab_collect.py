"""Tables of tools/ab.sh / tools/mid_ab.sh outputs (gpurun_out/ab_<tag>/*.log) for profiles/:
one row per (library, run): merges/s and the bench's per-kernel replay averages.

  python tools/ab_collect.py <out_dir> <tag>...   -> <out_dir>/<tag>.txt"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(d):
    out = []
    for f in sorted(os.listdir(d)):
        if not f.endswith(".log"):
            continue
        line = next((x for x in open(os.path.join(d, f)) if x.startswith('{"metric"')), None)
        if line is None:
            out.append((f[:-4], "no bench line", {}))
            continue
        j = json.loads(line)
        k = {n: v.get("avg_us") for n, v in (j.get("kernels") or {}).items()}
        roof = j.get("roofline") or {}
        if roof.get("avg_launch_us") is not None:
            k.setdefault(roof.get("kernel", "roof"), roof.get("avg_launch_us"))
        for n, v in (j.get("roofline_other") or {}).items():
            if (v or {}).get("avg_launch_us") is not None:
                k.setdefault(n, v["avg_launch_us"])
        pp = (j.get("pair_count_pass") or {}).get("pass_and_pack") or {}
        if pp.get("time_us") is not None:  # (the bin pass + k_pack, once per run, outside the timed merges)
            k["pass+pack"] = pp["time_us"]
        out.append((f[:-4], j["value"], k))
    return out


def main():
    dst, tags = sys.argv[1], sys.argv[2:]
    os.makedirs(dst, exist_ok=True)
    for t in tags:
        src = os.path.join(REPO, "gpurun_out", f"ab_{t}")
        with open(os.path.join(dst, f"{t}.txt"), "w") as f:
            f.write("# library.run  merges/s  per-kernel average launch (us, bench replay)\n")
            for name, v, k in rows(src):
                ks = " ".join(f"{n}={u}" for n, u in k.items() if u is not None)
                f.write(f"{name:24s} {v}  {ks}\n")


if __name__ == "__main__":
    main()
