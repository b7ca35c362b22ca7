"""CPU: the C-ABI library loads, exports every entry point include/kge_hip.h
declares, its ctypes mirror has the C layout (checked against gcc on the
header itself), and descriptor validation reports the reference's errors
without touching a GPU."""

import ctypes
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kge_hip.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(kge_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib(hiplib):
    return hiplib


def test_every_declared_symbol_is_exported(lib):
    from KGE import _hip
    names = _declared_functions()
    assert "kge_step" in names and "kge_sample" in names
    for n in names:
        assert hasattr(lib, n), "libkge_hip.so does not export %s" % n
    assert set(names) == set(_hip.EXPORTS)


def test_abi_version(lib):
    from KGE import _hip
    assert lib.kge_abi_version() == _hip.ABI_VERSION


def _c_layout():
    """offsetof / sizeof of every ABI struct, compiled by gcc from the header."""
    from KGE import _hip
    structs = {"kge_table": _hip.kge_table, "kge_sampler_desc": _hip.kge_sampler_desc,
               "kge_sample_desc": _hip.kge_sample_desc, "kge_step_desc": _hip.kge_step_desc}
    for extra in ("kge_apply_desc", "kge_rank_desc", "kge_apply_rows_desc", "kge_stream_desc", "kge_exchange_desc",
                  "kge_exchange_rows_desc"):
        if hasattr(_hip, extra):
            structs[extra] = getattr(_hip, extra)
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "kge_hip.h"', 'int main(void){']
    for s, cls in structs.items():
        lines.append('printf("%s sizeof %%zu\\n", sizeof(%s));' % (s, s))
        for f, _ in cls._fields_:
            lines.append('printf("%s %s %%zu\\n", offsetof(%s, %s));' % (s, f, s, f))
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "layout.c")
        exe = os.path.join(d, "layout")
        open(c, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(HEADER), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    return structs, {tuple(l.split()[:2]): int(l.split()[2]) for l in out.splitlines()}


def test_ctypes_mirror_matches_c_layout():
    structs, lay = _c_layout()
    for s, cls in structs.items():
        assert ctypes.sizeof(cls) == lay[(s, "sizeof")], s
        for f, _ in cls._fields_:
            assert getattr(cls, f).offset == lay[(s, f)], (s, f)


def _desc(**kw):
    from KGE import _hip
    d = _hip.kge_step_desc()
    d.abi_version = _hip.ABI_VERSION
    d.model = _hip.MODEL_TRANSE
    buf = (ctypes.c_float * 64)()
    addr = ctypes.addressof(buf)
    d.ent = _hip.kge_table(addr, 10, 4, 4)
    d.rel = _hip.kge_table(addr, 3, 4, 4)
    d.dim = 4
    d.pos = addr
    d.batch = 2
    d.negative_ratio = 2
    d.corrupt_side = _hip.SIDE_HT
    d.sampler.kind = _hip.SAMPLER_UNIFORM
    d.sampler.n_entities = 10
    d.score_kind = 0
    d.score_p = 2.0
    d.loss_kind = 0
    d.margin = 1.0
    d.optimizer = _hip.OPT_SGD
    d.lr = 0.01
    d.clip_norm = 5.0
    d.loss_out = addr
    for k, v in kw.items():
        setattr(d, k, v)
    return d, buf


def test_workspace_query_valid_descriptor(lib):
    d, _keep = _desc()
    assert lib.kge_step_workspace_bytes(ctypes.byref(d)) > 0


@pytest.mark.parametrize("field,value,status,msg", [
    ("corrupt_side", 7, 1, "Invalid corrupt_side"),
    ("abi_version", 99, 1, "abi_version"),
    ("loss_kind", 9, 1, "loss kind"),
    ("dim", 5, 1, "columns"),
    ("score_p", -1.0, 1, "p > 0"),
    ("negative_ratio", -1, 1, "negative_ratio"),
])
def test_invalid_descriptors_are_rejected_without_gpu(lib, field, value, status, msg):
    d, _keep = _desc(**{field: value})
    assert lib.kge_step_workspace_bytes(ctypes.byref(d)) == 0
    assert lib.kge_step(ctypes.byref(d), None) == status
    assert msg in lib.kge_last_error().decode()


def test_small_workspace_is_rejected(lib):
    d, _keep = _desc()
    need = lib.kge_step_workspace_bytes(ctypes.byref(d))
    ws = (ctypes.c_uint8 * 16)()
    d.workspace = ctypes.addressof(ws)
    d.workspace_bytes = 16
    assert need > 16
    assert lib.kge_step(ctypes.byref(d), None) == 4   # KGE_ENOMEM_WORKSPACE


def test_python_status_mapping():
    """kge_status -> the reference's exception types (ValueError for its asserts /
    InvalidArgument, NotImplementedError for unsupported fused combos)."""
    from KGE import _hip
    _hip.load()
    with pytest.raises(ValueError):
        _hip.check(_hip.KGE_EINVAL, "x")
    with pytest.raises(NotImplementedError):
        _hip.check(_hip.KGE_EUNSUPPORTED, "x")
    with pytest.raises(RuntimeError):
        _hip.check(_hip.KGE_EHIP, "x")
