"""C-ABI checks that need no GPU: the library loads, exports every symbol declared in
include/bo_amd.h, and the pure host-side helpers behave (no kernels are launched)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "bo_amd.h")).read()
    return sorted(set(re.findall(r"\b(bo_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from bayesopt_smart_amd import _lib
    lib = _lib.load()
    declared = _declared()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) <= set(_lib.symbols())


def test_status_strings_and_version():
    from bayesopt_smart_amd import _lib
    lib = _lib.load()
    assert lib.bo_abi_version() == _lib.ABI_VERSION == 5
    assert lib.bo_status_string(_lib.ERR_NOT_PD) == b"Matrix is not positive definite"
    with pytest.raises(np.linalg.LinAlgError):
        _lib.check(_lib.ERR_SINGULAR, "x")
    with pytest.raises(_lib.BoNativeError):
        _lib.check(_lib.ERR_ARG, "x")


def test_desc_layout_matches_header():
    """ctypes mirror of bo_predict_desc has the C layout (checked against offsetof via a
    tiny C program compiled with gcc)."""
    import subprocess
    import tempfile
    from bayesopt_smart_amd import _lib
    fields = [f for f, _ in _lib.PredictDesc._fields_]
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"bo_amd.h\"\nint main(){\n"
    prog += 'printf("%zu\\n", sizeof(bo_predict_desc));\n'
    for f in fields:
        prog += f'printf("%zu\\n", offsetof(bo_predict_desc, {f}));\n'
    prog += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        vals = [int(v) for v in subprocess.check_output([exe]).split()]
    assert vals[0] == ctypes.sizeof(_lib.PredictDesc)
    for f, off in zip(fields, vals[1:]):
        assert getattr(_lib.PredictDesc, f).offset == off, f
    # bo_sobol_desc likewise
    sf = [f for f, _ in _lib.SobolDesc._fields_]
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"bo_amd.h\"\nint main(){\n"
    prog += 'printf("%zu\\n", sizeof(bo_sobol_desc));\n'
    for f in sf:
        prog += f'printf("%zu\\n", offsetof(bo_sobol_desc, {f}));\n'
    prog += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        vals = [int(v) for v in subprocess.check_output([exe]).split()]
    assert vals[0] == ctypes.sizeof(_lib.SobolDesc)
    for f, off in zip(sf, vals[1:]):
        assert getattr(_lib.SobolDesc, f).offset == off, f


def test_workspace_size_queries():
    from bayesopt_smart_amd import _lib
    lib = _lib.load()
    d = _lib.PredictDesc()
    d.n_obj, d.dim, d.n_train, d.n_cand, d.cand_kind, d.topq = 2, 2, 512, 1 << 20, _lib.CAND_GRID, 3
    d.grid_shape[0] = d.grid_shape[1] = 1024
    ws = lib.bo_predict_workspace_size(d)
    assert ws >= 2 * 512 * 512 * 8
    d.topq = 49
    assert lib.bo_predict_workspace_size(d) == 0          # over BO_MAX_TOPQ
    d.topq, d.n_obj = 3, 9
    assert lib.bo_predict_workspace_size(d) == 0          # over BO_MAX_OBJ
    assert lib.bo_select_topq_workspace_size(1000, 3) > 0


def test_device_code_sha_identifies_the_kernels(tmp_path):
    """bench.py's PMC matching key: the sha256 of the library's .hip_fatbin section (every gfx950
    code object).  It exists for the in-tree library, it is the section llvm-objcopy dumps, and a
    file without that section (here: the library's host part only) has none."""
    import shutil
    import subprocess
    import sys
    sys.path.insert(0, ROOT)
    import hashlib
    from bench import device_code_sha256
    from bayesopt_smart_amd import _lib
    sha = device_code_sha256(_lib.LIB_PATH)
    assert sha is not None and re.fullmatch(r"[0-9a-f]{64}", sha)
    objcopy = "/opt/rocm/llvm/bin/llvm-objcopy"
    if os.path.exists(objcopy):
        dump = tmp_path / "fatbin.bin"
        subprocess.run([objcopy, f"--dump-section=.hip_fatbin={dump}", _lib.LIB_PATH, str(tmp_path / "x.so")],
                       check=True, capture_output=True)
        assert hashlib.sha256(dump.read_bytes()).hexdigest() == sha
        host = tmp_path / "host.so"
        subprocess.run([objcopy, "--remove-section=.hip_fatbin", _lib.LIB_PATH, str(host)], check=True,
                       capture_output=True)
        assert device_code_sha256(str(host)) is None
    not_elf = tmp_path / "not_elf.bin"
    shutil.copyfile(os.path.join(ROOT, "README.md"), not_elf)
    assert device_code_sha256(str(not_elf)) is None
