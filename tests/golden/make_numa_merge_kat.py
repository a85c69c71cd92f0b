"""Transcribe the topology-manager merge tests of the reference into tests/golden/numa_merge_kat.json.

Source (read as text): pkg/scheduler/frameworkext/topologymanager/policy_test.go —
commonPolicyMergeTestCases (:60), bestEffortPolicy.mergeTestCases (:344, also used by the Restricted
policy test, policy_restricted_test.go:71-79) and singleNumaNodePolicy.mergeTestCases (:612); numaNodes
= [0, 1] in every Merge test. Run from the repo root with the reference mounted; the JSON it writes is
the committed fixture (data only).
"""
import json
import re
import sys

SRC = "/root/reference/pkg/scheduler/frameworkext/topologymanager/policy_test.go"


def parse_hint_list(txt):
    out = []
    for m in re.finditer(r"NUMANodeAffinity:\s*(NewTestBitMask\(([\d, ]*)\)|nil),\s*Preferred:\s*(true|false)", txt):
        bits = None if m.group(1) == "nil" else [int(x) for x in m.group(2).split(",") if x.strip()]
        out.append([bits, m.group(3) == "true"])
    return out


def parse_provider(txt):
    body = txt.strip()
    if body in ("", "{}") or "map[string][]NUMATopologyHint" not in body:
        return None                       # &mockNUMATopologyHintProvider{} → nil map
    inner = body[body.index("map[string][]NUMATopologyHint") + len("map[string][]NUMATopologyHint"):]
    res = {}
    for m in re.finditer(r'"(\w+)":\s*(nil|\{)', inner):
        if m.group(2) == "nil":
            res[m.group(1)] = None
            continue
        start = m.end() - 1
        depth, i = 0, start
        while True:
            if inner[i] == "{":
                depth += 1
            elif inner[i] == "}":
                depth -= 1
                if depth == 0:
                    break
            i += 1
        res[m.group(1)] = parse_hint_list(inner[start:i + 1])
    return res


def split_providers(hp):
    provs, i = [], 0
    key = "&mockNUMATopologyHintProvider{"
    while True:
        j = hp.find(key, i)
        if j < 0:
            return provs
        k = j + len(key) - 1
        depth = 0
        while True:
            if hp[k] == "{":
                depth += 1
            elif hp[k] == "}":
                depth -= 1
                if depth == 0:
                    break
            k += 1
        provs.append(parse_provider(hp[j + len(key):k]))
        i = k


def cases_in(block, policies):
    out = []
    for c in re.split(r"\n\t\t\{\n\t\t\tname:\s*", block)[1:]:
        name = re.match(r'"([^"]*)"', c).group(1)
        hp_m = re.search(r"hp:\s*\[\]NUMATopologyHintProvider\{(.*?)\n\t\t\t\},?\n\t\t\texpected", c, re.S)
        hp = hp_m.group(1) if hp_m else ""
        exp = re.search(r"expected:\s*NUMATopologyHint\{\s*NUMANodeAffinity:\s*(NewTestBitMask\(([^)]*)\)|nil),\s*"
                        r"Preferred:\s*(true|false)", c)
        if exp.group(1) == "nil":
            bits = None
        elif exp.group(2).strip() == "numaNodes...":
            bits = [0, 1]
        else:
            bits = [int(x) for x in exp.group(2).split(",") if x.strip()]
        out.append({"name": name, "policies": policies, "providers": split_providers(hp),
                    "want": {"mask": bits, "preferred": exp.group(3) == "true"}})
    return out


def main():
    src = open(SRC).read()
    a = src.index("func commonPolicyMergeTestCases")
    b = src.index("func (p *bestEffortPolicy) mergeTestCases")
    c = src.index("func (p *singleNumaNodePolicy) mergeTestCases")
    d = src.index("func testPolicyMerge")
    cases = cases_in(src[a:b], ["BestEffort", "Restricted", "SingleNUMANode"])
    cases += cases_in(src[b:c], ["BestEffort", "Restricted"])
    cases += cases_in(src[c:d], ["SingleNUMANode"])
    doc = {"source": "pkg/scheduler/frameworkext/topologymanager/policy_test.go:60-883 (reference @ 2025-01-12)",
           "numa_nodes": [0, 1], "cases": cases}
    json.dump(doc, open(sys.argv[1] if len(sys.argv) > 1 else "tests/golden/numa_merge_kat.json", "w"), indent=1)
    print(len(cases), "cases")


if __name__ == "__main__":
    main()
