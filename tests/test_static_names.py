"""Every name a function of the host-side Python reads resolves: to its own scope, an enclosing
one, the module's globals or a builtin (symtable, no import of the file).  Catches a name left in
one function after an edit that belongs to another's scope -- bench.py's config-4 workload once
called main()'s nested finish_gather and failed only at run time, on the GPU box."""
import builtins
import glob
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = ["bench.py", "__graft_entry__.py"] + sorted(
    os.path.relpath(f, ROOT) for f in glob.glob(os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd", "**", "*.py"),
                                                recursive=True))


def _undefined(path):
    src = open(os.path.join(ROOT, path)).read()
    top = symtable.symtable(src, path, "exec")
    module_names = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()
                    or s.is_namespace()}
    known = module_names | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__", "__path__"}
    if "*" in {s.get_name() for s in top.get_symbols()}:
        return []
    bad = []

    def walk(t):
        for s in t.get_symbols():
            if s.is_global() and not s.is_declared_global() and s.is_referenced() and s.get_name() not in known:
                bad.append(f"{t.get_name()}:{s.get_name()}")
        for c in t.get_children():
            walk(c)

    walk(top)
    return bad


@pytest.mark.parametrize("path", FILES)
def test_no_undefined_names(path):
    assert _undefined(path) == []
