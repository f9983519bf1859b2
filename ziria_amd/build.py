"""Builds libziria_rx.so (all HIP kernels + the C-ABI) in-tree for gfx950 with hipcc.

The library is the product: ziria_amd's Python layer only loads it.  Output:
ziria_amd/_lib/libziria_rx.so (git-ignored, travels to the GPU box with the snapshot).
Translation units: zrx_api.hip (kernels, device API, batched externals; hipcc for gfx950),
zrx_host.cpp (the per-call externals on the host CPU, AVX2) and zrx_ext_cxx.cpp (the
externals with the C++ linkage wplc output links against), the last two with g++.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIBDIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIBDIR, "libziria_rx.so")


def source_hash():
    """sha256 over the kernel sources and the C-ABI header (name + content, sorted): ties a
    PMC summary in profiles/ to the kernels it was measured on (bench.py traffic fields)."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".h", ".py", ".cpp")))
    for f in files:
        h.update(f.encode())
        h.update(open(os.path.join(CSRC, f), "rb").read())
    h.update(open(os.path.join(HERE, "..", "include", "ziria_rx.h"), "rb").read())
    return h.hexdigest()[:16]


HOST_SRCS = ("zrx_host.cpp", "zrx_ext_cxx.cpp")   # host-only TUs, g++


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(HERE, "..", "include", "ziria_rx.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


DRIVER = os.path.join(LIBDIR, "ziria_rx_driver")
DRIVER_SRC = [os.path.join(HERE, "..", "tools", "ziria_rx_driver.cpp"),
              os.path.join(HERE, "..", "integration", "csrc", "hip_ext_batch.cpp")]


PERCALL = os.path.join(LIBDIR, "percall_bench")
PERCALL_SRC = [os.path.join(HERE, "..", "tools", "percall_bench.cpp")]


def _host_tool(exe, srcs, verbose):
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(max(os.path.getmtime(s) for s in srcs),
                                                            os.path.getmtime(LIB)):
        return exe
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(HERE, "..", "include"), "-o", exe + ".tmp"] + \
        list(srcs) + ["-L" + LIBDIR, "-lziria_rx", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(exe + ".tmp", exe)
    return exe


def build_driver(verbose=False):
    """The host programs linked against the library (rpath $ORIGIN, next to it in
    ziria_amd/_lib): the standalone batching driver (tools/ziria_rx_driver.cpp around the
    driver.cpp hook of integration/csrc/hip_ext_batch.cpp) and the per-call bench
    (tools/percall_bench.cpp)."""
    _host_tool(PERCALL, PERCALL_SRC, verbose)
    return _host_tool(DRIVER, DRIVER_SRC, verbose)


def build(force=False, verbose=False):
    if not force and not _stale():
        build_driver(verbose)
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    subprocess.check_call([sys.executable, os.path.join(CSRC, "gen_tables.py")])
    objs = []
    for src in HOST_SRCS:
        obj = os.path.join(LIBDIR, os.path.splitext(src)[0] + ".o")
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wextra", "-c", "-o", obj,
               os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd, cwd=CSRC)
        objs.append(obj)
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-pthread", "-o", LIB + ".tmp", os.path.join(CSRC, "zrx_api.hip"), "-x", "none"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(LIB + ".tmp", LIB)
    build_driver(verbose)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
