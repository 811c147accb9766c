"""List every `from VAESNe.<module> import <names>` line of the reference's cannon/
scripts (read as text; nothing is imported or executed) into cannon_imports.json,
the drop-in contract tests/test_boundary_cpu.py checks against the build.

    python tests/golden/gen_cannon_imports.py [/root/reference/cannon]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PAT = re.compile(r"^\s*from\s+VAESNe\.(\w+)\s+import\s+([\w ,]+?)\s*(?:#.*)?$", re.M)


def scan(root):
    out = []
    for d, _, files in os.walk(root):
        for f in sorted(files):
            if not f.endswith(".py"):
                continue
            path = os.path.join(d, f)
            src = open(path, encoding="utf-8", errors="replace").read()
            for m in PAT.finditer(src):
                line = src.count("\n", 0, m.start()) + 1
                for name in m.group(2).split(","):
                    out.append({"script": os.path.relpath(path, os.path.dirname(root)),
                                "line": line, "module": m.group(1), "name": name.strip()})
    return sorted(out, key=lambda e: (e["script"], e["line"], e["name"]))


if __name__ == "__main__":
    root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/cannon"
    entries = scan(root)
    with open(os.path.join(HERE, "cannon_imports.json"), "w") as fh:
        json.dump(entries, fh, indent=1)
    print(f"{len(entries)} imports from {len({e['script'] for e in entries})} scripts")
