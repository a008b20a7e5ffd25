"""Build libmms2ut_hip.so (gfx950) in-tree with hipcc: one object per csrc/*.hip, linked shared.

    python multimodal-s2ut_amd/build.py [--force]

The .so lands in multimodal-s2ut_amd/lib/ (git-ignored, travels to the GPU box with gpurun)."""
import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
LIB = os.path.join(LIBDIR, "libmms2ut_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall", "-Wno-unused-function",
         "-munsafe-fp-atomics", f"-I{INCLUDE}"]


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _deps_mtime():
    ts = [os.path.getmtime(os.path.join(CSRC, f)) for f in os.listdir(CSRC)]
    ts += [os.path.getmtime(os.path.join(INCLUDE, f)) for f in os.listdir(INCLUDE)]
    ts.append(os.path.getmtime(__file__))
    return max(ts)


def _headers_mtime():
    ts = [os.path.getmtime(os.path.join(CSRC, f)) for f in os.listdir(CSRC) if f.endswith(".h")]
    ts += [os.path.getmtime(os.path.join(INCLUDE, f)) for f in os.listdir(INCLUDE)]
    ts.append(os.path.getmtime(__file__))
    return max(ts)


def _compile(src, force=True):
    """-> (object path, True if hipcc ran)"""
    obj = os.path.join(OBJDIR, src.replace(".hip", ".o"))
    if not force and os.path.exists(obj) and \
            os.path.getmtime(obj) >= max(os.path.getmtime(os.path.join(CSRC, src)), _headers_mtime()):
        return obj, False      # object newer than its source and every header: reuse
    cmd = [HIPCC, *FLAGS, "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj, True


def build(force=False, verbose=True):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= _deps_mtime():
        if verbose:   # one line either way, so a build check can tell a rebuild from an up-to-date tree
            print(f"build: {LIB} up to date (newer than all {len(srcs)} csrc/*.hip sources, headers and "
                  f"build.py); --force recompiles", file=sys.stderr)
        return LIB
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        res = list(ex.map(lambda f: _compile(f, force), srcs))
    objs = [o for o, _ in res]
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(tmp, LIB)
    if verbose:
        done = [s for s, (_, ran) in zip(srcs, res) if ran]
        print(f"build: hipcc --offload-arch={ARCH} compiled {len(done)} of {len(srcs)} sources "
              f"({', '.join(done) or 'none'}), linked {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    build(force=ap.parse_args().force)
