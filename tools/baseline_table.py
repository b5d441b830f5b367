"""Rebuild profiles/baseline_configs.md's measured tables from bench/baseline_configs.py
JSON lines. Usage: python tools/baseline_table.py NEW.jsonl PREV.jsonl > table.md"""
import json
import sys


def load(path):
    out = {}
    with open(path) as fh:
        for line in fh:
            line = line.strip()
            if line.startswith("{"):
                d = json.loads(line)
                out[d["config"]] = d
    return out


def main():
    new, prev = load(sys.argv[1]), load(sys.argv[2])
    print("| config | ms / fit (median) | samples/s | nodes | depth | engine | previous ms |")
    print("|---|---:|---:|---:|---:|---|---:|")
    for k, d in new.items():
        if "engine" not in d or d["engine"] in ("cpu-native", "hip-small"):
            continue
        p = prev.get(k, {}).get("ms_median")
        print(f"| {k} | {d['ms_median']:.2f} | {d.get('samples_per_sec', 0) / 1e6:.1f}M | "
              f"{d['nodes']} | {d.get('depth', '')} | {d['engine']} | "
              f"{'' if p is None else f'{p:.2f}'} |")
    print()
    print("| n | ours 1x MI355X ms | ours CPU ms |")
    print("|---:|---:|---:|")
    for k, d in new.items():
        if k.startswith("sweep_gpu_n="):
            n = k.split("=")[1]
            c = new.get(f"sweep_n={n}", {}).get("ms_median")
            print(f"| {n} | {d['ms_median']:.3f} | {'' if c is None else f'{c:.3f}'} |")


if __name__ == "__main__":
    main()
