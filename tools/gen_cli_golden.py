"""Generate tests/golden/cli_flags.json from the REFERENCE main.py's argparse surface.

Reads /root/reference/main.py as text and walks its syntax tree (ast; nothing is
imported or executed: the file needs TensorFlow): the per-step tables `steps`,
`entity_nodes`, `hunk_nodes`, `entity_edges`, `hunk_edges` (main.py:11-15) and every
`parser.add_argument(...)` call inside the step loop (main.py:24-48).  A default that
names a loop variable (`default=entity_node`, main.py:39-45) is resolved per step from
the zipped tables, as the loop does.  Only the resulting flag table is committed: per
step, the flag, dest, type name, default and help string in call order.

Run from the repo root:  python tools/gen_cli_golden.py
"""
import ast
import json
import os

REF = "/root/reference/main.py"
TABLES = ("steps", "entity_nodes", "hunk_nodes", "entity_edges", "hunk_edges")


def _literal(node):
    return ast.literal_eval(node)


def main():
    tree = ast.parse(open(REF, encoding="utf-8").read())
    fn = next(n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == "main")
    tables = {}
    for st in fn.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1 and \
                isinstance(st.targets[0], ast.Name) and st.targets[0].id in TABLES:
            tables[st.targets[0].id] = _literal(st.value)
    loop = next(n for n in fn.body if isinstance(n, ast.For))
    loop_vars = [e.id for e in loop.target.elts]          # step, entity_node, ...
    calls = [n for n in ast.walk(loop) if isinstance(n, ast.Call)
             and isinstance(n.func, ast.Attribute) and n.func.attr == "add_argument"]
    calls.sort(key=lambda c: (c.lineno, c.col_offset))
    rows = list(zip(*(tables[t] for t in TABLES)))
    out = []
    for row in rows:
        env = dict(zip(loop_vars, row))
        flags = []
        for c in calls:
            flag = _literal(c.args[0])
            kw = {k.arg: k.value for k in c.keywords}
            if "default" in kw:
                d = kw["default"]
                default = env[d.id] if isinstance(d, ast.Name) else _literal(d)
            else:
                default = None
            flags.append({
                "flag": flag,
                "dest": _literal(kw["dest"]) if "dest" in kw else flag.lstrip("-"),
                "type": kw["type"].id if "type" in kw else None,
                "default": default,
                "help": _literal(kw["help"]) if "help" in kw else None,
                "line": c.lineno,
            })
        out.append({"step": env, "flags": flags})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tests", "golden", "cli_flags.json")
    with open(path, "w") as f:
        json.dump({"tables": tables, "loop_vars": loop_vars, "per_step": out,
                   "generator": "tools/gen_cli_golden.py",
                   "reference": "main.py @ fanmengdan/HD-GNN 2025-03-01 (ast walk, not executed)"},
                  f, indent=1)
    print("%d steps x %d flags -> %s" % (len(out), len(calls), path))


if __name__ == "__main__":
    main()
