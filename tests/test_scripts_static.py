"""The probe scripts against today's binding, statically (CPU, no GPU call).

VERDICT r04 found probe scripts that drove kernel forms since removed.  Every
script under scripts/ must at least compile and name only what the binding
still has: every `tcpck.<name>` it reads exists in tcp-stack_amd/tcpck, and
every method it calls on a context exists on tcpck.Context.  (Which kernel
variant numbers a library accepts is checked on the GPU by the variant tests.)
"""
import ast
import glob
import os
import py_compile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = sorted(glob.glob(os.path.join(ROOT, "scripts", "*.py")))
CTX_NAMES = {"ctx", "c", "pctx", "c0", "c1", "ctx0", "ctx1"}


@pytest.mark.parametrize("path", SCRIPTS, ids=[os.path.basename(p) for p in SCRIPTS])
def test_script_names_exist(path):
    import tcpck
    py_compile.compile(path, doraise=True)
    tree = ast.parse(open(path).read(), path)
    missing = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Attribute) and isinstance(node.value, ast.Name):
            if node.value.id in ("tcpck", "K") and not hasattr(tcpck, node.attr):
                missing.add(f"tcpck.{node.attr}")
            if node.value.id in CTX_NAMES and isinstance(getattr(node, "ctx", None), ast.Load):
                if not node.attr.startswith("_") and not hasattr(tcpck.Context, node.attr):
                    missing.add(f"Context.{node.attr}")
    assert not missing, f"{os.path.basename(path)} names what the binding no longer has: {sorted(missing)}"
