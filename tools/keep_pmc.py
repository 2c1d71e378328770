#!/usr/bin/env python3
"""Copy the sf:: kernel rows of every p_counter_collection.csv (and of the
kernel traces / stats of a ``trace`` pass) under a pmc_passes.sh output tree
(gpurun_out/...) into profiles/<name>/ (same relative paths), dropping
torch's own kernels, plus the library.json the passes recorded.

    python tools/keep_pmc.py gpurun_out/r2z_prof profiles/round2z_pmc c4eval c4 ...
"""
import os
import sys


KEEP = ("p_counter_collection.csv", "t_kernel_trace.csv", "t_kernel_stats.csv")


def main():
    src, dst, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
    for sub in subs:
        for root, _, files in os.walk(os.path.join(src, sub)):
            for f in files:
                if f == "library.json":  # the library the passes ran on
                    rel = os.path.relpath(os.path.join(root, f), src)
                    os.makedirs(os.path.dirname(os.path.join(dst, rel)), exist_ok=True)
                    open(os.path.join(dst, rel), "w").write(open(os.path.join(root, f)).read())
                    continue
                if f not in KEEP:
                    continue
                rel = os.path.relpath(os.path.join(root, f), src)
                lines = open(os.path.join(root, f)).read().splitlines()
                keep = [lines[0]] + [x for x in lines[1:] if 'sf::' in x]
                os.makedirs(os.path.dirname(os.path.join(dst, rel)), exist_ok=True)
                open(os.path.join(dst, rel), "w").write("\n".join(keep) + "\n")
                print(rel, len(keep) - 1)


if __name__ == "__main__":
    main()
