"""Generates tests/golden/numa_policy.json: the topology-manager Merge vectors of the reference
(pkg/scheduler/frameworkext/topologymanager/policy_test.go commonPolicyMergeTestCases / mergeTestCases, run by
policy_{best_effort,restricted,single_numa_node}_test.go with numaNodes = [0, 1]; policy_none_test.go
TestPolicyNoneMerge) and the IterateBitMasks cases of pkg/util/bitmask/bitmask_test.go.

The Go composite literals of the test tables are read from the reference test files (run in the container that has
/root/reference; the output JSON is the committed fixture) and turned into data: each case's providers (resource
name -> hint list, nil list or empty list) and the expected hint (mask bits or nil, preferred).

    python tests/golden/make_golden_policy.py
"""
import json
import os
import re

REF = "/root/reference/pkg/scheduler/frameworkext/topologymanager"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "numa_policy.json")
NUMA_NODES = [0, 1]

TOK = re.compile(r'\s*(?:(//[^\n]*)|("(?:[^"\\]|\\.)*")|(\.\.\.)|([A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z_][A-Za-z0-9_]*)*)|(-?\d+)|([{}()\[\],:&*]))')


def tokenize(text):
    pos, out = 0, []
    while pos < len(text):
        m = TOK.match(text, pos)
        if not m:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"cannot tokenize at {text[pos:pos + 40]!r}")
        pos = m.end()
        if m.group(1):
            continue
        out.append(next(g for g in m.groups()[1:] if g is not None))
    return out


class Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        if want is not None and tok != want:
            raise ValueError(f"expected {want!r}, got {tok!r} at token {self.i}")
        self.i += 1
        return tok

    def type_expr(self):
        # []T, map[string][]T, *T, pkg.T
        parts = []
        while self.peek() in ("[", "]", "*") or (self.peek() and re.match(r"[A-Za-z_]", self.peek())):
            if self.peek() == "[":
                self.take("[")
                inner = "" if self.peek() == "]" else self.take()
                self.take("]")
                parts.append(f"[{inner}]")
            else:
                parts.append(self.take())
            if parts[-1] not in ("*",) and not parts[-1].startswith("[") and self.peek() != "[":
                break
        return "".join(parts)

    def value(self):
        tok = self.peek()
        if tok == "&":
            self.take("&")
            return self.value()
        if tok == "{":
            return self.composite(None)
        if tok.startswith('"'):
            return json.loads(self.take())
        if tok in ("true", "false"):
            return self.take() == "true"
        if tok == "nil":
            self.take()
            return None
        if re.fullmatch(r"-?\d+", tok):
            return int(self.take())
        if tok == "NewTestBitMask":
            self.take()
            self.take("(")
            bits = []
            while self.peek() != ")":
                a = self.take()
                if a == ",":
                    continue
                if a == "numaNodes":
                    self.take("...")
                    bits.extend(NUMA_NODES)
                else:
                    bits.append(int(a))
            self.take(")")
            return {"mask": bits}
        if tok in ("[", "map") or re.match(r"[A-Za-z_]", tok):
            typ = self.type_expr()
            if self.peek() == "{":
                return self.composite(typ)
            return {"ident": typ}
        raise ValueError(f"unexpected token {tok!r}")

    def composite(self, typ):
        self.take("{")
        elems = []
        while self.peek() != "}":
            if self.peek(1) == ":" and (self.peek().startswith('"') or re.match(r"[A-Za-z_]", self.peek())):
                k = self.take()
                k = json.loads(k) if k.startswith('"') else k
                self.take(":")
                elems.append((k, self.value()))
            else:
                elems.append((None, self.value()))
            if self.peek() == ",":
                self.take(",")
        self.take("}")
        return {"type": typ, "elems": elems}


def hint(v):
    if v is None:
        return None
    f = dict(v["elems"]) if v["elems"] and v["elems"][0][0] is not None else {}
    aff = f.get("NUMANodeAffinity")
    return {"mask": aff["mask"] if aff else None, "preferred": bool(f.get("Preferred", False))}


def provider(v):
    # &mockNUMATopologyHintProvider{} -> no hints (nil map); {map[string][]NUMATopologyHint{...}}
    if not v["elems"]:
        return None
    mp = v["elems"][0][1]
    if mp is None:
        return None
    return {k: (None if lst is None else [hint(h) for _, h in lst["elems"]]) for k, lst in mp["elems"]}


def cases_of(body_tokens):
    p = Parser(body_tokens)
    while p.peek() != "return":
        p.i += 1
    p.take("return")
    lit = p.value()
    out = []
    for _, c in lit["elems"]:
        f = dict(c["elems"])
        out.append({"name": f["name"], "providers": [provider(x) for _, x in f["hp"]["elems"]],
                    "expected": hint(f["expected"])})
    return out


def func_tokens(text, header):
    start = text.index(header)
    brace = text.index("{", start + len(header) - 1)
    depth, i = 0, brace
    while True:
        if text[i] == "{":
            depth += 1
        elif text[i] == "}":
            depth -= 1
            if depth == 0:
                break
        i += 1
    return tokenize(text[brace + 1:i]), text[:start].count("\n") + 1


def main():
    src = open(os.path.join(REF, "policy_test.go")).read()
    groups = {}
    for key, header in (("common", "func commonPolicyMergeTestCases(numaNodes []int) []policyMergeTestCase {"),
                        ("best_effort", "func (p *bestEffortPolicy) mergeTestCases(numaNodes []int) []policyMergeTestCase {"),
                        ("single_numa_node", "func (p *singleNumaNodePolicy) mergeTestCases(numaNodes []int) []policyMergeTestCase {")):
        toks, line = func_tokens(src, header)
        cs = cases_of(toks)
        for c in cs:
            c["src"] = f"frameworkext/topologymanager/policy_test.go:{line} ({key})"
        groups[key] = cs
    out = {
        "numa_nodes": NUMA_NODES,
        # which case groups each policy's Merge test runs (policy_*_test.go:53-60, 71-78, 159-166)
        "runs": {"best_effort": ["common", "best_effort"], "restricted": ["common", "best_effort"],
                 "single_numa_node": ["common", "single_numa_node"]},
        "cases": groups,
        # policy_none_test.go:70-130: Merge returns an empty hint and admits
        "none_expected": {"mask": None, "preferred": False, "admit": True},
        # bitmask_test.go:583-633: IterateBitMasks over bits 0..n-1 visits 2^n - 1 masks
        "iterate_bitmasks_counts": {str(n): (1 << n) - 1 for n in (1, 2, 4, 8, 16)},
    }
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT, {k: len(v) for k, v in groups.items()})


if __name__ == "__main__":
    main()
