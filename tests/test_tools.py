"""Developer tooling kept honest on the CPU: every timing build of tools/diag_variant.py (a phase
removed from a scratch copy of csrc/) still applies to the product source, and the
product source carries no diagnostic switch."""
import importlib.util
import os
import re

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(ROOT, "npe-pfn_amd", "csrc")


def _diag():
    spec = importlib.util.spec_from_file_location("diag_variant", os.path.join(ROOT, "tools", "diag_variant.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_every_diag_edit_matches_the_source():
    for name, edits in _diag().EDITS.items():
        for fn, old, _new in edits:
            src = open(os.path.join(CSRC, fn)).read()
            assert src.count(old) >= 1, (name, fn, old[:60])


def test_no_diagnostic_switch_in_the_product_source():
    for fn in os.listdir(CSRC):
        src = open(os.path.join(CSRC, fn)).read()
        assert not re.search(r"NPFN_(IA_)?DIAG_", src), fn
