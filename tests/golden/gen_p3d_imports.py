"""Lists every ``from pytorch3d... import name`` in the reference's Python files into
tests/golden/p3d_imports.json (data: module -> names), for tests/test_p3d_shim.py.
Runs only in the build container (reads /root/reference as text)."""
import ast
import glob
import json
import os

REF = "/root/reference"
out = {}
for f in sorted(glob.glob(os.path.join(REF, "**", "*.py"), recursive=True)):
    for node in ast.walk(ast.parse(open(f).read())):
        if isinstance(node, ast.ImportFrom) and node.module and node.module.startswith("pytorch3d"):
            out.setdefault(node.module, set()).update(a.name for a in node.names)
json.dump({k: sorted(v) for k, v in sorted(out.items())},
          open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "p3d_imports.json"), "w"), indent=1)
print({k: len(v) for k, v in out.items()})
