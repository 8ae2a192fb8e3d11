"""Build libcsmom.so from another source tree (a git worktree of an earlier commit) into a given
path, with __graft_entry__'s flags, for same-box A/B runs through CSMOM_LIB:
    git worktree add /tmp/base <commit>
    python scripts/build_variant.py /tmp/base ab/libcsmom_base.so
    CSMOM_LIB=ab/libcsmom_base.so python bench.py ...
EXTRA_FLAGS="-DNAME=value ..." adds compile definitions (a variant of the same tree)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as G  # noqa: E402

src_root = Path(sys.argv[1]).resolve()
out = Path(sys.argv[2]).resolve()
csrc = src_root / G.CSRC.relative_to(G.ROOT)
srcs = [csrc / p.name for p in G.SRCS]
objdir = out.parent / (out.stem + "_obj")
objdir.mkdir(parents=True, exist_ok=True)
cflags = [f for f in G.FLAGS if f != "-shared"] + os.environ.get("EXTRA_FLAGS", "").split()


def cc(src):
    subprocess.run([G.HIPCC, *cflags, "-c", "-o", str(objdir / (src.stem + ".o")), str(src)],
                   check=True)


with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
    list(ex.map(cc, srcs))
subprocess.run([G.HIPCC, *G.FLAGS, "-o", str(out), *[str(objdir / (s.stem + ".o")) for s in srcs]],
               check=True)
print("built", out)
