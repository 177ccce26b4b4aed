"""Time variant libraries (lib/variants/libjpgx_NAME.so; "product" = lib/libjpgx.so) on the bench
workload with fresh input (8 x 4K q90, two input sets alternating, settled 300 ms): HIP-event
us per launch (min / median of 5 x 20), fraction of 8 TB/s at 9 B/px, and whether the output
of frame set 0 equals the product library's.  One process per library, interleaved rounds.
Usage (GPU box): python tools/kbench.py [ROUNDS] name ..."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kbench_child.py")


def lib_path(n):
    if n == "product":
        return os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "libjpgx.so")
    return os.path.join(REPO, "jpeg-encoder-and-decoder_amd", "lib", "variants", f"libjpgx_{n}.so")


def main():
    args = sys.argv[1:]
    rounds = int(args.pop(0)) if args and args[0].isdigit() else 2
    names = args
    sr = int(os.environ.get("KB_SUB", "0"))
    bpp = 9 if sr == 0 else (7 if sr == 1 else 6)
    res = {}
    for _ in range(rounds):
        for n in ["product"] + [x for x in names if x != "product"]:
            env = dict(os.environ, JPGX_LIB=lib_path(n))
            r = subprocess.run([sys.executable, CHILD], env=env, capture_output=True,
                               text=True, timeout=300)
            if r.returncode:
                print(n, "ERROR", r.stderr[-400:], flush=True)
                continue
            res.setdefault(n, []).append(json.loads(r.stdout.strip().splitlines()[-1]))
            d = res[n][-1]
            print(f"{n:12s} min {d['us'][0]:7.1f} us  med {d['us'][2]:7.1f}  frac(min) "
                  f"{8 * 3840 * 2160 * bpp / (d['us'][0] * 1e-6) / 8e12:.4f}  "
                  f"same-as-product={d['hash'] == res['product'][0]['hash']}", flush=True)


if __name__ == "__main__":
    main()
