"""The C-ABI library loads and exports every symbol include/ptsharp_hip.h declares;
argument validation and error reporting work without a GPU (no compute calls)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from ptsharp_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ptsharp_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pt_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = declared_functions()
    for n in ["pt_create", "pt_upload_scene", "pt_render_pass", "pt_read_buffer", "pt_stats_get", "pt_last_error",
              "pt_destroy", "pt_comm_unique_id", "pt_comm_init", "pt_comm_gather"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = _abi.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(_abi.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported with C linkage"


def test_version():
    assert _abi.load_library().pt_get_version() == _abi.ABI_VERSION


def test_struct_layouts_match_header():
    # sizes computed by hand from the C declarations (x86-64 SysV alignment)
    assert C.sizeof(_abi.pt_mesh_data) == 8 + 9 * 8
    assert C.sizeof(_abi.pt_material) == 8 * 8 + 6 * 4 + 8
    assert C.sizeof(_abi.pt_texture) == 16
    assert C.sizeof(_abi.pt_camera) == 12 * 4 + 3 * 8
    assert C.sizeof(_abi.pt_sampler) == 24
    assert C.sizeof(_abi.pt_pass_params) == 4 + 4 + 8 + 4 + 4 + 8 + 8 + 8 + 4 + 4   # passes, tail padding
    assert C.sizeof(_abi.pt_stats) == 9 * 8 + 8 * 8 + 8 * 4 + 8 + 8   # + tail_handoffs (ABI 9)
    assert C.sizeof(_abi.pt_trace_counters) == 88 + 8 * 8   # + march_clock[8] (ABI 8)
    assert _abi.pt_scene_desc.env_color.offset % 8 == 0


def test_null_arguments_rejected_with_message():
    lib = _abi.load_library()
    assert lib.pt_create(None, None) == _abi.PT_ERR_INVALID_ARG
    assert b"NULL" in lib.pt_last_error()
    assert lib.pt_upload_scene(None, None) == _abi.PT_ERR_INVALID_ARG
    assert lib.pt_render_pass(None, None, None, None) == _abi.PT_ERR_INVALID_ARG
    assert lib.pt_read_buffer(None, None, None, None) == _abi.PT_ERR_INVALID_ARG
    assert lib.pt_stats_get(None, None) == _abi.PT_ERR_INVALID_ARG
    assert lib.pt_comm_gather(None, 0) == _abi.PT_ERR_INVALID_ARG
    lib.pt_destroy(None)  # no-op


def test_bad_dimensions_rejected():
    lib = _abi.load_library()
    ctx = C.c_void_p()
    opts = _abi.pt_device_opts(0, 1, 1)
    assert lib.pt_create(C.byref(opts), C.byref(ctx)) == _abi.PT_ERR_INVALID_ARG
    assert not ctx.value


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_device_reports_error_not_fallback():
    lib = _abi.load_library()
    ctx = C.c_void_p()
    opts = _abi.pt_device_opts(0, 64, 64)
    rc = lib.pt_create(C.byref(opts), C.byref(ctx))
    assert rc in (_abi.PT_ERR_NO_DEVICE, _abi.PT_ERR_HIP)
    assert lib.pt_last_error()
    from ptsharp_amd import Renderer, scenes
    s, c, smp = scenes.furnace()
    with pytest.raises(_abi.PTError):
        Renderer.NewRenderer(s, c, smp, 64, 64, True)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        _abi.load_library(str(tmp_path / "missing.so"))


# canonical field types: C (include/ptsharp_hip.h), C# (csharp/HipRenderer.cs), ctypes (_abi.py)
_C_TYPES = {"int32_t": "i32", "int": "i32", "uint32_t": "u32", "uint64_t": "u64", "double": "f64", "float": "f32",
            "uint8_t": "u8"}
_CS_TYPES = {"int": "i32", "uint": "u32", "ulong": "u64", "long": "i64", "double": "f64", "float": "f32",
             "byte": "u8", "IntPtr": "ptr"}


def _macros(src):
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (\w+) (\d+)", src)}


def _fields_c(src, name):
    """[(field, type, length)] of a typedef struct in the header (pointer fields: type 'ptr')."""
    macros = _macros(src)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    out = []
    for decl in body.split(";"):
        decl = " ".join(decl.replace("const ", "").split())
        if not decl:
            continue
        base, names = decl.split(None, 1)
        base_ptr = base.endswith("*")
        base = base.rstrip("*")
        for n in names.split(","):
            n = n.strip()
            ptr = base_ptr or n.startswith("*")
            m = re.match(r"\*?\s*(\w+)(?:\[(\w+)\])?", n)
            ln = m.group(2)
            ln = 1 if ln is None else int(ln) if ln.isdigit() else macros[ln]
            out.append((m.group(1), "ptr" if ptr else _C_TYPES[base], ln))
    return out


def _fields_cs(src, name):
    body = re.search(r"struct %s\s*\{(.*?)\}" % name, src, re.S).group(1)
    body = re.sub(r"//[^\n]*", "", body)
    out = []
    for decl in body.split(";"):
        decl = decl.replace("public", "").replace("fixed", "").replace("@", "").strip()
        if not decl:
            continue
        base, names = decl.split(None, 1)
        for n in names.split(","):
            m = re.match(r"\s*(\w+)(?:\[(\d+)\])?", n)
            out.append((m.group(1), _CS_TYPES[base], int(m.group(2) or 1)))
    return out


def _ctype_name(t):
    if isinstance(t, type) and issubclass(t, C._Pointer) or t in (C.c_void_p, C.c_char_p):
        return "ptr"
    return {C.c_int32: "i32", C.c_uint32: "u32", C.c_uint64: "u64", C.c_int64: "i64", C.c_double: "f64",
            C.c_float: "f32", C.c_uint8: "u8"}[t]


@pytest.mark.parametrize("name", ["pt_pass_params", "pt_stats", "pt_mesh_data", "pt_sampler", "pt_device_opts",
                                  "pt_camera", "pt_material", "pt_texture", "pt_scene_desc", "pt_sdf_node",
                                  "pt_sdf_shape", "pt_volume_window", "pt_volume", "pt_transformed_shape",
                                  "pt_trace_counters"])
def test_csharp_binding_matches_header(name):
    """csharp/HipRenderer.cs mirrors include/ptsharp_hip.h field for field: names, types (a float /
    double drift would corrupt the P/Invoke) and array lengths (the library writes pt_stats into the
    caller's struct, so a stale C# layout would be overrun)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    c = _fields_c(open(HEADER).read(), name)
    cs = _fields_cs(open(os.path.join(root, "csharp", "HipRenderer.cs")).read(), name)
    assert cs == c


@pytest.mark.parametrize("name", ["pt_pass_params", "pt_stats", "pt_mesh_data", "pt_sampler", "pt_device_opts",
                                  "pt_camera", "pt_material", "pt_texture", "pt_scene_desc", "pt_sdf_node",
                                  "pt_sdf_shape", "pt_volume_window", "pt_volume", "pt_transformed_shape",
                                  "pt_trace_counters"])
def test_python_binding_matches_header(name):
    """ptsharp_amd/_abi.py mirrors include/ptsharp_hip.h field for field (names, types, array lengths)."""
    c = _fields_c(open(HEADER).read(), name)
    py = []
    for fname, ftype in getattr(_abi, name)._fields_:
        n = getattr(ftype, "_length_", 1)
        py.append((fname, _ctype_name(ftype._type_ if n > 1 or hasattr(ftype, "_length_") else ftype), n))
    assert py == c


def test_csharp_declares_every_entry_point():
    """Every function of the header has a [DllImport] in the C# drop-in (multi-GPU included)."""
    cs = open(os.path.join(ROOT, "csharp", "HipRenderer.cs")).read()
    imported = set(re.findall(r"static extern \w+ (pt_\w+)\(", cs))
    assert imported == set(declared_functions())
