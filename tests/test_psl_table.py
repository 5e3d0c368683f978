"""The generated public suffix table (pktvisor_amd/csrc/pv_psl_data.h, written by tools/gen_psl.py)
against the reference's ICANN section, read here by a parser independent of gen_psl.py's
regular expressions, plus match_public_suffix sizes worked out by hand from the reference's
list (libs/visor_dns/PublicSuffixList.h:226-250). The device and the oracle compile the same
header, so GPU-vs-oracle parity cannot see a generator error; this test can."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "pktvisor_amd", "csrc", "pv_psl_data.h")
REF = "/root/reference/libs/visor_dns/PublicSuffixList.h"


def _c_strings(block: str):
    out = []
    for lit in re.findall(r'"((?:[^"\\]|\\[0-7]{3})*)"', block):
        b = bytearray()
        i = 0
        while i < len(lit):
            if lit[i] == "\\":
                b.append(int(lit[i + 1:i + 4], 8))
                i += 4
            else:
                b += lit[i].encode()
                i += 1
        out.append(bytes(b).decode("utf-8"))
    return out


def header_table():
    s = open(HDR, encoding="utf-8").read()
    tld = _c_strings(s.split("pv_psl_tld[PV_PSL_NTLD] = {", 1)[1].split("};", 1)[0])
    cnt = [int(x) for x in re.findall(r"\d+", s.split("pv_psl_count[PV_PSL_NTLD] = {", 1)[1].split("};", 1)[0])]
    sfx = _c_strings(s.split("pv_psl_sfx[PV_PSL_NSFX] = {", 1)[1].split("};", 1)[0])
    assert len(tld) == len(cnt) and sum(cnt) == len(sfx)
    table, k = [], 0
    for t, c in zip(tld, cnt):
        table.append((t, sfx[k:k + c]))
        k += c
    return table


def match_public_suffix(table, name: str) -> int:
    """PublicSuffixList.h:231-250 over the header's table (first key wins, as the map keeps it)"""
    pos = name.rfind(".")
    if pos < 0 or pos + 1 == len(name):
        return 0
    d = {}
    for k, v in table:
        d.setdefault(k, v)
    key = name[pos + 1:]
    if key not in d:
        return 0
    nb = name.encode()
    for s in d[key]:
        if nb.endswith(s.encode()):
            return len(s.encode()) + 1
    return len(key.encode()) + 1


def test_header_shape():
    t = header_table()
    assert len(t) == 200 and sum(len(v) for _, v in t) == 5840
    keys = [k for k, _ in t]
    assert len(set(keys)) == len(keys)
    d = dict(t)
    assert d["uk"][-1] == "*.sch.uk" and d["uk"][:2] == ["ac.uk", "co.uk"]
    assert d["us"].index("ak.us") < d["us"].index("k12.ak.us")
    assert "ac.za" in d and "za" not in d  # the reference's key holds a dot: unreachable by lookup


@pytest.mark.parametrize("name,size", [
    ("www.example.co.uk", 6),   # co.uk
    ("xco.uk", 6),              # byte suffix, not label: "xco.uk" ends with "co.uk"
    ("foo.sch.uk", 3),          # "*.sch.uk" is a literal: only the key "uk"
    ("a.*.sch.uk", 9),          # ... which a literal '*' label matches
    ("x.y.k12.ak.us", 6),       # "ak.us" is listed before "k12.ak.us": first listed match wins
    ("foo.ac.za", 0),           # no "za" key
    ("www.公司.香港", 14),       # IDN: byte length of "公司.香港" + 1
    ("example.jp", 3),          # key only
    ("uk", 0), ("foo.uk.", 0), ("host.invalidtld", 0),
])
def test_match_sizes_by_hand(name, size):
    assert match_public_suffix(header_table(), name) == size


@pytest.mark.skipif(not os.path.exists(REF), reason="reference tree absent (GPU box)")
def test_header_equals_reference_icann_section():
    """A line-oriented read of the reference's ICANN_DOMAINS initializer (each `{"key"sv, {...}},`
    entry on its own line), independent of gen_psl.py's regular expressions."""
    text = open(REF, encoding="utf-8").read()
    body = text.split("===BEGIN ICANN DOMAINS===", 1)[1].split("===END ICANN DOMAINS===", 1)[0]
    ref, seen = [], set()
    for line in body.splitlines():
        line = line.strip()
        if not line.startswith('{"'):
            continue
        key, rest = line[2:].split('"sv, {', 1)
        items = [x.strip() for x in rest.rsplit("}}", 1)[0].split(",") if x.strip()]
        vals = []
        for x in items:
            assert x.startswith('"') and x.endswith('"sv'), x
            vals.append(x[1:-3])
        if key in seen:
            continue
        seen.add(key)
        ref.append((key, vals))
    assert header_table() == ref
