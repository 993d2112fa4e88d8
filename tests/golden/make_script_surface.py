"""Extract the surface the reference's own scripts use into tests/golden/script_surface.json.

Reads /root/reference/scripts/{train,test,play,high_level_play}.py as text (``ast``; nothing of the reference is
imported or run) and records, per script: every import (module, imported names), the ``logger.*`` attributes, the
``Cfg.<group>.<field>`` paths, the attributes of the other imported names (``AC_Args._update`` ...), the
attributes read from ``env``, and the keyword names of the calls the scripts make
into the framework (VelocityTrackingEasyEnv, HistoryWrapper, Runner, runner.learn, ActorCritic).
tests/test_script_surface.py checks that every one of them resolves in this repository.
usage: python tests/golden/make_script_surface.py [reference_root]"""
import ast
import json
import os
import sys

SCRIPTS = ["train", "test", "play", "high_level_play"]
CALLS = {"VelocityTrackingEasyEnv", "HistoryWrapper", "Runner", "ActorCritic", "learn", "load_state_dict"}


def _chain(node):
    """a.b.c -> ["a", "b", "c"] for an Attribute chain rooted at a Name (else None)."""
    parts = []
    while isinstance(node, ast.Attribute):
        parts.append(node.attr)
        node = node.value
    if isinstance(node, ast.Name):
        return [node.id] + parts[::-1]
    return None


def surface(path):
    tree = ast.parse(open(path).read(), filename=path)
    imports, logger_attrs, cfg_paths, env_attrs, calls = [], set(), set(), set(), {}
    imported = {a.asname or a.name for n in ast.walk(tree) if isinstance(n, ast.ImportFrom) for a in n.names}
    class_attrs = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Import):
            for a in node.names:
                imports.append({"module": a.name, "names": []})
        elif isinstance(node, ast.ImportFrom) and node.level == 0:
            imports.append({"module": node.module, "names": [a.name for a in node.names]})
        elif isinstance(node, ast.Attribute):
            ch = _chain(node)
            if not ch:
                continue
            if ch[0] == "logger" and len(ch) >= 2:
                logger_attrs.add(ch[1])
            elif ch[0] == "Cfg" and len(ch) >= 3:
                cfg_paths.add(".".join(ch[1:3]))
            elif ch[0] == "env" and len(ch) >= 2:
                env_attrs.add(ch[1])
            elif ch[0] in imported and ch[0] != "Cfg" and len(ch) >= 2:
                class_attrs.setdefault(ch[0], set()).add(ch[1])
        if isinstance(node, ast.Call):
            f = node.func
            name = f.id if isinstance(f, ast.Name) else (f.attr if isinstance(f, ast.Attribute) else None)
            if name in CALLS:
                calls.setdefault(name, set()).update(k.arg for k in node.keywords if k.arg)
    uniq = {json.dumps(i, sort_keys=True) for i in imports}
    return {"imports": [json.loads(u) for u in sorted(uniq)], "logger_attrs": sorted(logger_attrs),
            "cfg_paths": sorted(cfg_paths), "env_attrs": sorted(env_attrs),
            "call_kwargs": {k: sorted(v) for k, v in sorted(calls.items())},
            "class_attrs": {k: sorted(v) for k, v in sorted(class_attrs.items())}}


def cfg_fields(path):
    """group.field for every field of the reference's Cfg (legged_robot_config.py: class Cfg's nested classes), and
    group._update for each group (params_proto's PrefixProto method)."""
    tree = ast.parse(open(path).read(), filename=path)
    out = set()
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == "Cfg":
            for grp in node.body:
                if isinstance(grp, ast.ClassDef):
                    out.add(f"{grp.name}._update")
                    for st in grp.body:
                        if isinstance(st, ast.Assign):
                            out.update(f"{grp.name}.{t.id}" for t in st.targets if isinstance(t, ast.Name))
                        elif isinstance(st, ast.ClassDef):
                            out.add(f"{grp.name}.{st.name}")
    return sorted(out)


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {s: surface(os.path.join(ref, "scripts", s + ".py")) for s in SCRIPTS}
    out["_reference_cfg_fields"] = cfg_fields(os.path.join(ref, "mini_gym", "envs", "base", "legged_robot_config.py"))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "script_surface.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", dst)


if __name__ == "__main__":
    main()
