#!/usr/bin/env python3
"""Build the in-tree native extension `_dfs_native` for gfx950.

Every source in csrc/ is compiled by hipcc (host C++ and HIP device code alike) with
`--offload-arch=gfx950` and linked against the HIP runtime, RCCL and OpenSSL. The .so is
written INSIDE the package so it travels with the repo snapshot to the GPU box.

    python build_native.py            # incremental
    python build_native.py --clean    # full rebuild
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
PKG = ROOT / "rust_hadoop_generated_by_llm_amd"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950").split(";")[0] or "gfx950"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.environ.get("HIPCC", f"{ROCM}/bin/hipcc")
# nghttp2 (native gRPC server): headers ship with the image's conda tree, the runtime library
# with the system; link the system soname so the extension loads without conda on the path
NGHTTP2_INC = os.environ.get("NGHTTP2_INC", "/opt/conda/include")
NGHTTP2_LIB = os.environ.get("NGHTTP2_LIB", "/usr/lib/x86_64-linux-gnu/libnghttp2.so.14")


def ext_path() -> Path:
    return PKG / ("_dfs_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def _includes() -> list[str]:
    import pybind11

    return [f"-I{CSRC}", f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
            f"-I{ROCM}/include"]


def _nghttp2_include() -> list[str]:
    """Only nghttp2's own headers (a copy under build/): putting the whole conda include
    directory on the path would shadow the system OpenSSL headers."""
    import shutil

    dst = BUILD / "nghttp2_include" / "nghttp2"
    if not (dst / "nghttp2.h").exists():
        dst.mkdir(parents=True, exist_ok=True)
        for f in ("nghttp2.h", "nghttp2ver.h"):
            shutil.copy2(Path(NGHTTP2_INC) / "nghttp2" / f, dst / f)
    return [f"-I{dst.parent}"]


def _newer(src: Path, obj: Path, headers: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


def build(clean: bool = False, verbose: bool = False) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    # native proto3 codec generated from proto/dfs.proto (no protoc in this toolchain)
    sys.path.insert(0, str(ROOT / "scripts"))
    import gen_proto

    gen_proto.main()
    sources = sorted(list(CSRC.glob("*.cpp")) + list(CSRC.glob("*.hip")))
    headers = sorted(CSRC.glob("*.h"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", "-fvisibility=hidden",
             f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__"] + _includes()
    jobs = []
    objs = []
    for src in sources:
        obj = BUILD / (src.name + ".o")
        objs.append(obj)
        if clean or _newer(src, obj, headers):
            lang = ["-x", "hip"] if src.suffix == ".hip" else []
            extra = _nghttp2_include() if src.name in ("grpc_server.cpp", "grpc_client.cpp") else []
            jobs.append([HIPCC, *flags, *extra, *lang, "-c", str(src), "-o", str(obj)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return cmd[-3]

    workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8"))) or 1
    with cf.ThreadPoolExecutor(workers) as ex:
        for name in ex.map(run, jobs):
            if verbose:
                print("built", name, flush=True)
    out = ext_path()
    if clean or not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
        link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", str(out), *map(str, objs),
                f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-lssl", "-lcrypto", NGHTTP2_LIB,
                "-lpthread", f"-Wl,-rpath,{ROCM}/lib"]
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    build_tools(objs, flags, clean, headers)
    if os.environ.get("DFS_BUILD_SANITIZERS", "1") == "1":
        build_sanitized(clean=clean)
    return out


def build_tools(objs: list[Path], flags: list[str], clean: bool, headers: list[Path]) -> list[Path]:
    """Native executables linked against the runtime objects: the benchmarks and unit tests
    (csrc/bench/*.cpp, e.g. io_bench) and the command-line tools (csrc/tools/*.cpp, dfs_cli).
    Written to build/native/ (ships to the GPU box)."""
    runtime = [o for o in objs if not o.name.startswith("bindings")]
    outs = []
    for src in sorted((CSRC / "bench").glob("*.cpp")) + sorted((CSRC / "tools").glob("*.cpp")):
        obj = BUILD / ("bench_" + src.name + ".o")
        exe = BUILD / src.stem
        if clean or _newer(src, obj, headers):
            r = subprocess.run([HIPCC, *flags, "-c", str(src), "-o", str(obj)], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
        if clean or not exe.exists() or any(o.stat().st_mtime > exe.stat().st_mtime for o in [obj, *runtime]):
            r = subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-o", str(exe), str(obj), *map(str, runtime),
                                f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", "-lrocprofiler-sdk-roctx", "-lssl", "-lcrypto",
                                NGHTTP2_LIB, "-lpthread", f"-Wl,-rpath,{ROCM}/lib"], capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed: {exe}\n{r.stdout}\n{r.stderr}")
        outs.append(exe)
    return outs


# Host-only runtime sources the native unit tests need (no HIP): they also build with the
# host compiler under ASan/UBSan and TSan (SURVEY §5.2 — the reference has no sanitizer runs).
SANITIZE_SOURCES = ["json.cpp", "json_dump.cpp", "shard_map.cpp", "raft.cpp", "wal.cpp", "crc32.cpp", "gf256.cpp",
                    "disk_gate.cpp", "extent_alloc.cpp", "master_core.cpp", "http_lite.cpp",
                    "journal.cpp", "audit_log.cpp", "lin_checker.cpp", "sts.cpp", "crypto.cpp", "tls.cpp",
                    "sigv4.cpp", "p2p_socket.cpp", "grpc_server.cpp", "grpc_client.cpp", "md5_mb.cpp"]
SANITIZERS = {"asan": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
              "tsan": ["-fsanitize=thread"]}


def build_sanitized(kinds=("asan", "tsan"), clean: bool = False) -> list[Path]:
    """build/native/unit_tests_<kind>: the native unit tests + host runtime under a sanitizer
    (host clang++, -O1 -g). GPU code never gets sanitizer instrumentation."""
    outs = []
    srcs = [CSRC / n for n in SANITIZE_SOURCES] + [CSRC / "bench" / "unit_tests.cpp"]
    headers = sorted(CSRC.glob("*.h"))
    for kind in kinds:
        exe = BUILD / f"unit_tests_{kind}"
        newest = max(p.stat().st_mtime for p in srcs + headers)
        if clean or not exe.exists() or exe.stat().st_mtime < newest:
            # LLVM's runtime (not GCC 11's) intercepts pthread_cond_clockwait, which libstdc++
            # uses for condition_variable::wait_for; without it TSan misreads every timed wait
            # host code only; roctx (trace.h), nghttp2 and OpenSSL are linked as shipped
            cmd = [f"{ROCM}/llvm/bin/clang++", "-std=c++17", "-O1", "-g", "-pthread", *SANITIZERS[kind],
                   f"-I{CSRC}", f"-I{ROCM}/include", *_nghttp2_include(), "-o", str(exe), *map(str, srcs),
                   f"-L{ROCM}/lib", "-lrocprofiler-sdk-roctx", "-lssl", "-lcrypto", NGHTTP2_LIB,
                   f"-Wl,-rpath,{ROCM}/lib"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"sanitizer build failed ({kind}):\n{r.stdout}\n{r.stderr}")
        outs.append(exe)
    return outs


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args()
    p = build(a.clean, a.verbose)
    print(p)
    sys.exit(0)
