"""INTEGRATION.md against the boundary header: the shim's pv_* calls type-check
against include/pvgpu.h (tests/integration_shim.cpp, compiled with g++ -fsyntax-only), and every
pv_* name the document mentions is declared there. CPU only."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_names():
    txt = open(os.path.join(ROOT, "include", "pvgpu.h")).read()
    return set(re.findall(r"\bpv_[a-z0-9_]+\b", txt))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_shim_calls_compile_against_header():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        os.path.join(ROOT, "tests", "integration_shim.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_integration_doc_names_exist():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    # (file names such as pv_bpf.cpp aside)
    named = set(re.findall(r"\bpv_[a-z0-9_]+\b(?![.](?:cpp|hip|h|py)\b)", doc))
    missing = sorted(n for n in named if n not in header_names())
    assert not missing, f"INTEGRATION.md names what include/pvgpu.h does not declare: {missing}"


def test_shim_covers_the_documented_shim_calls():
    # every pv_* call in the document's C++ blocks appears in the compiled stub
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = "\n".join(re.findall(r"```cpp\n(.*?)```", doc, re.S))
    blocks = re.sub(r"//[^\n]*", "", blocks)  # comments
    calls = set(re.findall(r"\b(pv_[a-z0-9_]+)\s*\(", blocks))
    stub = open(os.path.join(ROOT, "tests", "integration_shim.cpp")).read()
    missing = sorted(c for c in calls if not re.search(r"\b" + c + r"\s*\(", stub))
    assert not missing, f"shim calls not in tests/integration_shim.cpp: {missing}"
