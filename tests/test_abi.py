"""CPU-side checks of the drop-in boundary: the in-tree libfi_learner.so loads and exports every
function include/fi_learner.h declares; the product never imports the oracle."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(name="fi_learner.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fi_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from freeimpala_amd import _abi
    lib = _abi.lib()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_abi.SIGNATURES), set(names) ^ set(_abi.SIGNATURES)
    assert lib.fi_abi_version() == 1


def test_library_exports_every_farmer_header_symbol():
    """include/fi_farmer.h (the FarmerLstm train step) is exported by the same library."""
    from freeimpala_amd import farmer
    lib = farmer.lib()
    names = header_functions("fi_farmer.h")
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(farmer.SIGNATURES), set(names) ^ set(farmer.SIGNATURES)
    assert farmer.param_count() == 1_514_497  # the reference model's size


def test_farmer_struct_layouts_match_c():
    import ctypes
    import subprocess
    import tempfile
    from freeimpala_amd import farmer
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "fi_farmer.h"\nint main(){printf("%zu %zu %zu %zu",'
           'sizeof(fi_farmer_config), sizeof(fi_farmer_stats), offsetof(fi_farmer_config, device),'
           'offsetof(fi_farmer_stats, step));}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", os.path.join(d, "s")], check=True)
        out = subprocess.run([os.path.join(d, "s")], capture_output=True, text=True, check=True).stdout
    got = [int(v) for v in out.split()]
    exp = [ctypes.sizeof(farmer.FarmerConfig), ctypes.sizeof(farmer.FarmerStats),
           farmer.FarmerConfig.device.offset, farmer.FarmerStats.step.offset]
    assert got == exp


def test_struct_layouts_match_c():
    import ctypes
    import subprocess
    import tempfile
    from freeimpala_amd import _abi
    src = ('#include <stdio.h>\n#include <stddef.h>\n#include "fi_learner.h"\nint main(){printf("%zu %zu %zu %zu %zu",'
           'sizeof(fi_learner_config), sizeof(fi_step_stats), sizeof(fi_vtrace_hparams),'
           'offsetof(fi_learner_config, seed), offsetof(fi_learner_config, lr));}')
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", os.path.join(d, "s")], check=True)
        out = subprocess.run([os.path.join(d, "s")], capture_output=True, text=True, check=True).stdout
    got = [int(x) for x in out.split()]
    exp = [ctypes.sizeof(_abi.LearnerConfig), ctypes.sizeof(_abi.StepStats),
           ctypes.sizeof(_abi.VtraceHparams), _abi.LearnerConfig.seed.offset, _abi.LearnerConfig.lr.offset]
    assert got == exp


def test_product_never_imports_or_links_oracle():
    bad = []
    for d in ("freeimpala_amd", "include", "cmd"):
        base = os.path.join(ROOT, d)
        if not os.path.isdir(base):
            continue
        for dp, _, fs in os.walk(base):
            for f in fs:
                if f.endswith((".py", ".h", ".hip", ".cpp", ".c", ".hpp")):
                    txt = open(os.path.join(dp, f), errors="ignore").read()
                    if re.search(r"import\s+oracle|from\s+oracle|liboracle|orc_[a-z]", txt):
                        bad.append(os.path.join(dp, f))
    assert not bad, bad


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    import importlib
    from freeimpala_amd import _abi
    monkeypatch.setattr(_abi, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_abi, "_lib", None)
    import pytest
    with pytest.raises(_abi.FiError):
        _abi.lib()
    importlib.reload(_abi)
