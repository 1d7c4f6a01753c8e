"""Builds libsdl_batcher.so (HIP kernels + C ABI) in-tree for gfx950.

    python -m streaming_data_loader_amd.build      # or __graft_entry__.build()

Each translation unit is compiled with `hipcc --offload-arch=gfx950` into
build/, then linked into streaming_data_loader_amd/libsdl_batcher.so, which is
git-ignored but travels to the GPU box with the repo snapshot.  hipcc
cross-compiles without a GPU.
"""
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(REPO, "build", "sdl")
LIB = os.path.join(PKG, "libsdl_batcher.so")
ARCH = os.environ.get("SDL_OFFLOAD_ARCH", "gfx950")

SOURCES = ["tokenize_wordpiece.hip", "tokenize_bpe.hip", "tokenize_unigram.hip", "pipeline.hip", "json_text.hip", "transport_frame.hip", "inflate.hip",
           "assets.cpp", "sdl_batcher.cpp"]
HEADERS = ["common.hpp", "device_util.hpp", "kernels.hpp", "tok_device.hpp", "assets.hpp", "json.hpp", "unigram.hpp",
           "rows_device.hpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
         "-I", os.path.join(REPO, "include"), "-I", CSRC]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _newer(dst, srcs):
    if not os.path.exists(dst):
        return False
    t = os.path.getmtime(dst)
    return all(os.path.getmtime(s) <= t for s in srcs)


BUILD_ID_MARK = b"sdl-build-id:"


def source_hash(defines=()):
    """sha256 over the contents of every source, header and flag the library is
    built from -- what sdl_build_id() of an up-to-date library returns."""
    h = hashlib.sha256()
    for path in [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(REPO, "include", "sdl_batcher.h")]:
        h.update(os.path.basename(path).encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    h.update(" ".join(FLAGS[:-4] + [f"-D{d}" for d in defines]).encode())
    return h.hexdigest()


def embedded_id(lib):
    """The build id compiled into a library file (read from its bytes, no dlopen), or None."""
    try:
        with open(lib, "rb") as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(BUILD_ID_MARK)
    return data[i + len(BUILD_ID_MARK):i + len(BUILD_ID_MARK) + 64].decode("ascii", "replace") if i >= 0 else None


def build(verbose=False, force=False, jobs=4, defines=(), lib=None, build_dir=None):
    """defines: extra -D macros (diagnostic builds go to their own lib/build_dir).

    A library whose embedded build id equals source_hash() is used as is (the
    GPU box gets the library but not the objects: nothing is recompiled
    there); otherwise the changed objects are rebuilt and the id relinked."""
    lib = lib or LIB
    bdir = build_dir or BUILD
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    want = source_hash(defines)
    if not force and embedded_id(lib) == want:
        return lib
    hipcc = _hipcc()
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(REPO, "include", "sdl_batcher.h")]
    objs, todo = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(bdir, s + ".o")
        objs.append(obj)
        if force or not _newer(obj, [src] + hdrs):
            lang = ["-x", "hip"] if s.endswith(".hip") else []
            todo.append([hipcc] + FLAGS + [f"-D{d}" for d in defines] + lang + ["-c", src, "-o", obj])
    # the build id: a one-line translation unit regenerated per link
    idsrc = os.path.join(bdir, "build_id.cpp")
    with open(idsrc, "w") as f:
        f.write('extern "C" const char *sdl_build_id(void) {\n'
                f'    static const char id[] = "{BUILD_ID_MARK.decode()}{want}";\n'
                f'    return id + {len(BUILD_ID_MARK)};\n}}\n')
    idobj = idsrc + ".o"
    todo.append([hipcc, "-O2", "-fPIC", "-c", idsrc, "-o", idobj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        p = subprocess.run(cmd, capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{p.stdout}\n{p.stderr}")
        return p.stderr

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for err in ex.map(run, todo):
            if verbose and err:
                print(err, file=sys.stderr)
    run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib] + objs + [idobj, "-ldl"])
    if embedded_id(lib) != want:
        raise RuntimeError(f"{lib}: build id not embedded")
    return lib


def build_stamps():
    """Diagnostic build with per-phase s_memtime stamps -> var/stamps/libsdl_batcher.so (travels to the GPU box)."""
    return build(defines=("SDL_STAMPS=1",), lib=os.path.join(REPO, "var", "stamps", "libsdl_batcher.so"),
                 build_dir=os.path.join(REPO, "build", "stamps"))


GZ256_LIB = os.path.join(REPO, "var", "gz256", "libsdl_batcher.so")


def build_gz256():
    """Diagnostic build whose inflate output batch (256 B) cannot hold a 258-byte match, the
    r02 hang: the decoder must leave through its no-progress exit (GZ_E_STALL) instead ->
    var/gz256/libsdl_batcher.so (tests/test_inflate_fuzz.py::test_device_no_progress_exit)."""
    return build(defines=("SDL_GZ_OBUF=256", "SDL_GZ_ALLOW_SMALL_OBUF"), lib=GZ256_LIB,
                 build_dir=os.path.join(REPO, "build", "var", "gz256", "obj"))


def build_ablations(levels=(3,)):
    """Diagnostic load-only build of the WordPiece chunk kernel (SDL_ABLATE: the window and
    record bits staged, nothing tokenized) -> var/abl3/libsdl_batcher.so (tools/pmc_calibration.py)."""
    return [build(defines=(f"SDL_ABLATE={n}",), lib=os.path.join(REPO, "var", f"abl{n}", "libsdl_batcher.so"),
                  build_dir=os.path.join(REPO, "build", f"abl{n}")) for n in levels]


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
