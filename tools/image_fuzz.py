"""Fuzz rt_image_load against the reference's own loader (oracle/_ref, built by `make ref` where
/root/reference is present): for each seed, the whole tests/image_corpus.py corpus at a random picture size,
N mutated copies per file (truncation, random byte stores, header bit flips, random runs).  Criterion as
in tests/test_image_load.py: same success/failure and texels as stb's zero-initialised build, and as the
as-is build wherever stb's output does not depend on memory it never wrote.

    python tools/image_fuzz.py FIRST_SEED LAST_SEED [N=16]
"""
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
import image_corpus as corpus  # noqa: E402
from test_image_load import agrees_with_reference  # noqa: E402


def mutate(rng, data: bytes, kind: int) -> bytes:
    d = bytearray(data)
    if kind == 0:
        d = d[:int(rng.integers(0, len(d)))]
    elif kind == 1:
        for _ in range(int(rng.integers(1, 4))):
            d[int(rng.integers(0, len(d)))] = int(rng.integers(0, 256))
    elif kind == 2:
        d[int(rng.integers(0, min(len(d), 300)))] ^= 1 << int(rng.integers(0, 8))
    else:
        i = int(rng.integers(0, len(d)))
        j = min(len(d), i + int(rng.integers(1, 64)))
        d[i:j] = rng.integers(0, 256, j - i, dtype=np.uint8).tobytes()
    return bytes(d)


def main():
    first, last = int(sys.argv[1]), int(sys.argv[2])
    n_mut = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    tmp = Path(tempfile.mkdtemp(prefix="rt_imgfuzz_"))
    total = bad = uninit = 0
    t0 = time.time()
    for seed in range(first, last + 1):
        rng = np.random.default_rng(seed)
        files = corpus.corpus(seed, int(rng.integers(1, 40)), int(rng.integers(1, 60)))
        for name, data in files.items():
            for trial in range(n_mut):
                f = tmp / ("x." + name.rsplit(".", 1)[1])
                f.write_bytes(mutate(rng, data, trial % 4))
                ok, u = agrees_with_reference(f)
                total += 1
                uninit += u
                if not ok:
                    bad += 1
                    keep = tmp / f"bad_{seed}_{trial}_{name}"
                    keep.write_bytes(f.read_bytes())
                    print(f"MISMATCH seed {seed} {name} trial {trial}: {keep}", flush=True)
        print(f"seed {seed}: cumulative {total} files, {bad} mismatches, {uninit} uninit-dependent "
              f"({time.time() - t0:.0f} s)", flush=True)
    print(f"seeds {first}..{last}: {total} mutated files, {bad} mismatches, {uninit} where stb reads unwritten memory")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
