"""CPU: the C-ABI library loads and exports every entry point include/*.h
declares; layouts match the reference; no compute calls are made here (no
GPU in this container) except to prove the product fails loudly without one."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess
import sys

import pytest

import libhv_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def _declared_functions():
    names = set()
    for h in ("websocket_parser.h", "hvws.h", "hvws_synth.h", "wsdef.h"):
        src = open(os.path.join(INC, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        src = re.sub(r"static inline[^{]*\{.*?\n\}", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b([a-z_][a-z0-9_]*)\s*\(", src, flags=re.M):
            name = m.group(1)
            if name in ("if", "for", "while", "sizeof", "defined"):
                continue
            if src[m.start():m.end()].lstrip().startswith(("typedef", "#")):
                continue
            names.add(name)
    return names


def test_library_loads():
    L = libhv_amd.lib()
    assert os.path.exists(libhv_amd.LIB_PATH)
    assert L is libhv_amd.lib()


def test_every_declared_symbol_is_exported():
    L = libhv_amd.lib()
    names = _declared_functions()
    # the reference frame-layer ABI, by name (http/websocket_parser.h:70-90, http/wsdef.h)
    for must in ("websocket_parser_init", "websocket_parser_settings_init", "websocket_parser_execute",
                 "websocket_parser_decode", "websocket_decode", "websocket_calc_frame_size",
                 "websocket_build_frame", "ws_encode_key", "ws_calc_frame_size", "ws_build_frame",
                 "hvws_scan", "hvws_unmask", "hvws_step", "hvws_rx_batch", "hvws_pipeline", "hvws_synth"):
        assert must in names, must
    missing = [n for n in sorted(names) if not hasattr(L, n)]
    assert not missing, missing


def test_every_batch_entry_point_has_a_binding_signature():
    """The Python binding declares argtypes for every hvws_* entry point, so
    no pointer argument is ever passed through ctypes' default int conversion."""
    names = [n for n in _declared_functions() if n.startswith("hvws_")]
    missing = [n for n in sorted(names) if n not in libhv_amd._SIGS]
    assert not missing, missing


def test_cxx_drop_in_symbols_exported():
    out = subprocess.run(["nm", "-D", "--defined-only", libhv_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    for sym in libhv_amd.CXX_SYMBOLS:
        assert sym in out, sym


def test_struct_layouts_match_reference():
    # struct websocket_parser (http/websocket_parser.h:50-62) on x86-64 [probed]:
    # flags@4 mask@8 mask_offset@12 length@16 require@24 offset@32 data@40, 48 B
    P = libhv_amd.WsParser
    assert ctypes.sizeof(P) == 48
    assert [P.flags.offset, P.mask.offset, P.mask_offset.offset, P.length.offset, P.require.offset,
            P.offset.offset, P.data.offset] == [4, 8, 12, 16, 24, 32, 40]
    assert ctypes.sizeof(libhv_amd.Frame) == 40
    assert ctypes.sizeof(libhv_amd.Segment) == 16


def test_no_cpu_fallback_without_gpu():
    """With no usable device the receive path aborts with a diagnostic instead
    of silently computing on the CPU."""
    if libhv_amd.device_count() > 0:
        pytest.skip("a GPU is visible")
    code = (
        "import ctypes, libhv_amd\n"
        "L = libhv_amd.lib()\n"
        "p = libhv_amd.WsParser(); L.websocket_parser_init(ctypes.byref(p))\n"
        "s = (ctypes.c_void_p * 3)()\n"
        "d = bytes.fromhex('818537fa213d7f9f4d5158')\n"
        "L.websocket_parser_execute(ctypes.byref(p), s, d, len(d))\n"
        "print('RETURNED')\n"
    )
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "RETURNED" not in r.stdout
    assert "no CPU fallback" in r.stderr
    e = libhv_amd.lib().hvws_ctx_create(0)
    assert not e
    assert libhv_amd.lib().hvws_last_error()


def test_engine_errors_are_reported():
    with pytest.raises(libhv_amd.HvwsError):
        libhv_amd.Engine(0) if libhv_amd.device_count() == 0 else libhv_amd.Engine(10_000)


REF = "/root/reference"


@pytest.mark.skipif(not os.path.exists(os.path.join(REF, "http", "WebSocketParser.h")),
                    reason="reference headers only in the build container")
def test_builds_against_reference_headers(tmp_path):
    """libhv's callers compile against libhv's own headers.  tests/csrc/refabi.cpp
    is built against the reference's http/{WebSocketParser.h, websocket_parser.h,
    wsdef.h} (+ hexport.h) and against include/, each linked to libhvws.so with
    no undefined symbol allowed; the same static_asserts on the layouts pass in
    both; both programs print the same answers from the host-only entry
    points, which equal the reference library's."""
    src = os.path.join(ROOT, "tests", "csrc", "refabi.cpp")
    out = {}
    for name, inc in (("ref", [f"-I{REF}", f"-I{REF}/http"]), ("ours", [f"-I{INC}"])):
        exe = str(tmp_path / f"refabi_{name}")
        cmd = ["g++", "-std=c++11", "-O1", "-Wall", "-Werror", "-Wno-invalid-offsetof", *inc, src,
               f"-L{os.path.dirname(libhv_amd.LIB_PATH)}", "-lhvws",
               f"-Wl,-rpath,{os.path.dirname(libhv_amd.LIB_PATH)}", "-Wl,--no-undefined",
               "-Wl,--unresolved-symbols=report-all", "-o", exe]
        r = subprocess.run(cmd, capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        out[name] = r.stdout
    assert out["ref"] == out["ours"]
    lines = out["ref"].splitlines()
    assert lines[0] == "init 0 0 0 0 0 0 1" and lines[1] == "settings 1 1 1"
    assert lines[-1] == "sizes 48 24 80"
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import wsharness as H

    if H.have_ref():
        R = H.ref()
        R.websocket_calc_frame_size.restype = ctypes.c_size_t
        R.websocket_calc_frame_size.argtypes = [ctypes.c_int, ctypes.c_size_t]
        R.ws_calc_frame_size.restype = ctypes.c_int
        R.ws_calc_frame_size.argtypes = [ctypes.c_int, ctypes.c_bool]
        n = 0
        for ln in lines:
            f = ln.split()
            if f[0] == "calc":
                assert int(f[3]) == R.websocket_calc_frame_size(int(f[2]), int(f[1])), ln
                n += 1
            elif f[0] == "wscalc":
                assert (int(f[2]), int(f[3])) == (R.ws_calc_frame_size(int(f[1]), False),
                                                  R.ws_calc_frame_size(int(f[1]), True)), ln
                n += 1
        assert n == 43
