"""Build tuning variants of the product library in parallel (lss-carla_amd/variants/<name>.so).

  python scripts/build_variants.py o6=LSS_SPLAT_OCC=6 zf=LSS_SPLAT_ZFIRST=1

Each argument is name=define[,define...]; the variants carry every source of the product library,
built with build.command plus the -D knobs (experiment switches of csrc/*.hip).
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from lss_carla_amd import build
    vdir = os.path.join(build.HERE, "variants")
    os.makedirs(vdir, exist_ok=True)
    jobs = []
    for a in sys.argv[1:]:
        name, _, defs = a.partition("=")
        jobs.append((name, [d for d in defs.split(",") if d]))

    def one(job):
        name, defs = job
        out = os.path.join(vdir, f"{name}.so")
        r = subprocess.run(build.command(out, defs), capture_output=True, text=True)
        return name, r.returncode, (r.stdout + r.stderr)[-2000:]

    workers = max(1, min(len(jobs), (os.cpu_count() or 2) // 2))
    with ThreadPoolExecutor(workers) as ex:
        for name, rc, msg in ex.map(one, jobs):
            print(f"{name}: {'ok' if rc == 0 else 'FAILED'}", flush=True)
            if rc:
                sys.stderr.write(msg)
                sys.exit(1)


if __name__ == "__main__":
    main()
