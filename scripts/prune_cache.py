#!/usr/bin/env python3
"""Drop in-tree cache entries (.gt_cache/gt_mi355x/<key>) that no current build uses.

    python scripts/prune_cache.py            # runs __graft_entry__.build() (which prebuilds the GPU
                                             # tests' libraries too) + the sweep prebuilds with
                                             # GTMI_CACHE_LOG set, then deletes the rest
    python scripts/prune_cache.py --dry-run

Every call of gpurun sends the whole tree; libraries of superseded code generations only add to
it. The GPU tests, smoke() and bench.py need exactly what build() prebuilds.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SWEEPS = os.path.join(REPO, "scripts", "sweep_keep.txt")  # "<config> <variants>" lines to keep


def main():
    dry = "--dry-run" in sys.argv
    fd, log = tempfile.mkstemp(prefix="gtmi_keys_")
    os.close(fd)
    env = dict(os.environ, GTMI_CACHE_LOG=log)
    subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.build()"], cwd=REPO, env=env, check=True)
    if os.path.exists(SWEEPS):
        with open(SWEEPS) as f:
            for line in f:
                line = line.strip()
                if line and not line.startswith("#"):
                    cfg, variants = line.split(None, 1)
                    subprocess.run([sys.executable, "scripts/sweep.py", "--config", cfg, "--variants", variants,
                                    "--build-only"], cwd=REPO, env=env, check=True)
    with open(log) as f:
        keep = {ln.strip() for ln in f if ln.strip()}
    os.unlink(log)
    root = os.path.join(REPO, ".gt_cache", "gt_mi355x")
    gone = [k for k in os.listdir(root) if k not in keep]
    for k in gone:
        if not dry:
            shutil.rmtree(os.path.join(root, k))
    print(f"kept {len(keep)} entries, {'would delete' if dry else 'deleted'} {len(gone)}")


if __name__ == "__main__":
    main()
