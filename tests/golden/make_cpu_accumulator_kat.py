"""Transcribe NodeNUMAResource's cpuset-take tests into tests/golden/cpu_accumulator_kat.json.

Source (read as text): pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go — the table
tests TestTakeFullPCPUs (:59), TestTakeFullPCPUsWithNUMALeastAllocated (:175), TestTakeSpreadByPCPUs
(:301), TestTakeSpreadByPCPUsWithNUMALeastAllocated (:373) and TestTakeCPUsWithExclusivePolicy (:435),
whose takeCPUs call arguments per test function are listed in CALLS below; the sequential tests
TestTakeCPUsWithMaxRefCount (:560), TestTakeCPUsSortByRefCount (:601) and TestTakePreferredCPUs (:758)
are written out as steps (their expectations are the assert lines' cpusets).  Run from the repo root
with the reference mounted; the JSON it writes is the committed fixture (data only).
"""
import json
import re

SRC = "/root/reference/pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go"

# test function → (bind policy, exclusive policy, NUMA allocate strategy) of its takeCPUs call;
# None = the case's own field (TestTakeCPUsWithExclusivePolicy defaults: :538-543)
CALLS = {
    "TestTakeFullPCPUs": ("FullPCPUs", "None", "MostAllocated"),
    "TestTakeFullPCPUsWithNUMALeastAllocated": ("FullPCPUs", "None", "LeastAllocated"),
    "TestTakeSpreadByPCPUs": ("SpreadByPCPUs", "None", "MostAllocated"),
    "TestTakeSpreadByPCPUsWithNUMALeastAllocated": ("SpreadByPCPUs", "None", "LeastAllocated"),
    "TestTakeCPUsWithExclusivePolicy": (None, None, "MostAllocated"),
}


def parse_cpuset(txt):
    m = re.search(r'cpuset\.NewCPUSet\(([\d, ]*)\)', txt)
    if m:
        return sorted(int(x) for x in m.group(1).split(",") if x.strip())
    m = re.search(r'cpuset\.MustParse\("([^"]*)"\)', txt)
    out = []
    for part in filter(None, m.group(1).split(",")):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return sorted(out)


def field(body, name):
    m = re.search(r"\b" + name + r":\s*(.+?),\n", body)
    return None if m is None else m.group(1).strip()


def table_cases(src, func):
    start = src.index(f"func {func}(t *testing.T)")
    body = src[start:src.index("\n}\n", start)]
    cases = []
    for m in re.finditer(r"\{\n\s*name:\s*\"(.*?)\",\n(.*?)\n\t\t\},", body, flags=re.S):
        name, b = m.group(1), m.group(2) + "\n"
        topo = [int(x) for x in re.search(r"buildCPUTopologyForTest\((\d+), (\d+), (\d+), (\d+)\)", b).groups()]
        alloc_txt = field(b, "allocatedCPUs") or field(b, "allocatedExclusiveCPUs")
        bind, excl, strategy = CALLS[func]
        case = {"name": name, "test": func, "topology": topo, "max_ref": int(field(b, "maxRefCount")),
                "allocated": parse_cpuset(alloc_txt) if alloc_txt else [],
                "need": int(field(b, "numCPUsNeeded")), "want_error": field(b, "wantError") == "true",
                "want": parse_cpuset(field(b, "wantResult")), "strategy": strategy}
        if func == "TestTakeCPUsWithExclusivePolicy":
            pol = lambda f, d: (re.search(r"Policy(\w+)$", field(b, f)).group(1) if field(b, f) else d)
            case["allocated_exclusive"] = pol("allocatedExclusivePolicy", "PCPULevel")
            case["excl"] = pol("exclusivePolicy", "PCPULevel")
            case["bind"] = pol("bindPolicy", "SpreadByPCPUs")
        else:
            case["bind"], case["excl"] = bind, excl
            case["allocated_exclusive"] = ""
        cases.append(case)
    return cases


def main():
    src = open(SRC).read()
    table = []
    for func in CALLS:
        table += table_cases(src, func)
    # sequential tests: steps of (need, bind, want) on one node allocation with maxRefCount 2
    # (TestTakeCPUsWithMaxRefCount :560-599, TestTakeCPUsSortByRefCount :601-653; core ids remapped to
    # socket << 16 | core, every allocation added with exclusive policy PCPULevel)
    seq = [
        {"name": "TestTakeCPUsWithMaxRefCount", "topology": [1, 1, 4, 2], "max_ref": 2, "steps": [
            {"need": 4, "bind": "FullPCPUs", "want": [0, 1, 2, 3]},
            {"need": 5, "bind": "FullPCPUs", "want": [0, 4, 5, 6, 7]},
            {"need": 4, "bind": "FullPCPUs", "want": [2, 3, 4, 5]}]},
        {"name": "TestTakeCPUsSortByRefCount", "topology": [1, 1, 16, 2], "max_ref": 2, "steps": [
            {"need": 16, "bind": "SpreadByPCPUs", "want": list(range(0, 32, 2))},
            {"need": 16, "bind": "FullPCPUs", "want": list(range(16))},
            {"need": 16, "bind": "SpreadByPCPUs", "want": list(range(1, 32, 2))},
            {"need": 16, "bind": "FullPCPUs", "want": list(range(16, 32))}],
         "want_available_after": []},
    ]
    # TestTakePreferredCPUs (:758-777): topology (2, 1, 16, 2), SpreadByPCPUs, None, MostAllocated
    preferred = [
        {"available": "all", "preferred": None, "need": 2, "want": [0, 2]},
        {"available": "all", "preferred": [0, 2], "need": 2, "want": [0, 2]},
        {"available": "all-but-0,2", "preferred": [], "need": 2, "want": [1, 3]},
        {"available": "all", "preferred": [11, 13, 15, 17], "need": 2, "want": [11, 13]},
    ]
    # TestCPUSpreadByPCPUs (:291) / ...WithNUMALeastAllocated (:363): freeCPUs(false) + spreadCPUs on
    # (2, 2, 4, 2) with 8 needed — the order of the first pass (evens) then the odds
    spread = list(range(0, 32, 2)) + list(range(1, 32, 2))
    doc = {"source": "pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go", "table": table,
           "sequential": seq, "preferred": {"topology": [2, 1, 16, 2], "cases": preferred},
           "spread_order": {"topology": [2, 2, 4, 2], "want": spread}}
    with open("tests/golden/cpu_accumulator_kat.json", "w") as f:
        json.dump(doc, f, indent=1)
    print(len(table), "table cases")


if __name__ == "__main__":
    main()
