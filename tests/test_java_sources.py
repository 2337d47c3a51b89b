"""The Java drop-in (java/) against the C boundary it binds, checked without a JVM (the image has none):

- every StructLayout in SentinelGpu.java, member by member, has the offsets and size the C compiler
  gives the struct of include/sentinel_gpu.h (a C file listing offsetof() of each member is generated
  from the Java source and compiled with gcc), and each member is naturally aligned, as the FFM API
  requires of a struct layout;
- SentinelGpu.java has a downcall handle for every export of the header, and its constants are the
  header's;
- the ServiceLoader file names the builder class, which implements SlotChainBuilder;
- the JVM replay harness's input exporter (tools/jvm_replay.py) writes what the harness parses.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from sentinel_amd import _abi as A
from sentinel_amd import engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JAVA = os.path.join(ROOT, "java", "src", "main", "java", "com", "alibaba", "csp", "sentinel", "gpu")
if not os.path.isdir(JAVA):  # the java/ sources do not travel to the GPU box (.gpurunignore)
    pytest.skip("java/ sources absent", allow_module_level=True)
SG = open(os.path.join(JAVA, "SentinelGpu.java")).read()

_SIZE = {"JAVA_INT": 4, "JAVA_LONG": 8, "JAVA_DOUBLE": 8, "JAVA_SHORT": 2, "JAVA_BYTE": 1, "ADDRESS": 8}


def java_layouts():
    """{c_struct: [(member, offset, size, align)], size} from the structLayout blocks, FFM semantics:
    members are laid out back to back (no implicit padding), paddingLayout(n) is explicit."""
    out = {}
    for m in re.finditer(r"static final StructLayout (\w+) = MemoryLayout\.structLayout\((.*?)\)\.withName\(\"(\w+)\"\);",
                         SG, re.S):
        body, cname = m.group(2), m.group(3)
        off, members = 0, []
        for line in [x.strip().rstrip(",") for x in body.strip().splitlines()]:
            pad = re.fullmatch(r"MemoryLayout\.paddingLayout\((\d+)\)", line)
            seq = re.fullmatch(r"MemoryLayout\.sequenceLayout\((\d+), (\w+)\)\.withName\(\"(\w+)\"\)", line)
            val = re.fullmatch(r"(\w+)\.withName\(\"(\w+)\"\)", line)
            if pad:
                off += int(pad.group(1))
            elif seq:
                k, t, name = int(seq.group(1)), seq.group(2), seq.group(3)
                members.append((name, off, k * _SIZE[t], _SIZE[t]))
                off += k * _SIZE[t]
            elif val:
                t, name = val.group(1), val.group(2)
                members.append((name, off, _SIZE[t], _SIZE[t]))
                off += _SIZE[t]
            else:
                raise AssertionError("unparsed layout line in %s: %r" % (cname, line))
        out[cname] = (members, off)
    return out


def test_every_boundary_struct_has_a_java_layout():
    got = set(java_layouts())
    want = {"sg_config", "sg_flow_rule", "sg_degrade_rule", "sg_param_item", "sg_param_rule", "sg_event",
            "sg_event_ext", "sg_arg", "sg_metric_node", "sg_token_req", "sg_token_result", "sg_param_token_req"}
    assert want <= got, want - got


def test_java_layouts_match_the_c_compiler(tmp_path):
    lay = java_layouts()
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "%s"' % os.path.join(ROOT, "include", "sentinel_gpu.h"),
             "int main(void) {"]
    for s, (members, _) in lay.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (s, s))
        for name, *_ in members:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (s, name, s, name))
    lines += ["return 0;", "}"]
    src = tmp_path / "java_abi.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "java_abi"
    subprocess.run(["gcc", "-O0", "-o", str(exe), str(src)], check=True)
    c = {k: int(v) for k, v in (l.rsplit(" ", 1) for l in subprocess.run([str(exe)], capture_output=True,
                                                                         text=True, check=True).stdout.splitlines())}
    for s, (members, size) in lay.items():
        assert size == c[s], (s, size, c[s])
        for name, off, msize, align in members:
            assert off == c["%s.%s" % (s, name)], (s, name, off, c["%s.%s" % (s, name)])
            assert off % align == 0, (s, name, "misaligned: FFM would reject the layout")
        # FFM arrays of the struct need its size to be a multiple of its alignment
        assert size % max(a for *_, a in members) == 0, s
    # a few fields the Java side writes by name
    assert c["sg_config.aux_node_capacity"] == A.SgConfig.aux_node_capacity.offset
    assert c["sg_event.aux"] == A.EVENT_DTYPE.fields["aux"][1]


def test_every_export_has_a_downcall_handle():
    bound = set(re.findall(r'fn\("(sg_\w+)"', SG))
    assert bound == set(engine.EXPORTS), set(engine.EXPORTS) ^ bound


def test_java_constants_are_the_headers():
    def const(name):
        m = re.search(r"\b%s = (0x[0-9A-Fa-f]+L?|\d+)" % name, SG)
        assert m, name
        return int(m.group(1).rstrip("L"), 0)
    assert (const("EV_ENTRY"), const("EV_EXIT"), const("EV_TRACE")) == (A.EV_ENTRY, A.EV_EXIT, A.EV_TRACE)
    assert (const("F_PRIORITIZED"), const("F_HAS_ARG"), const("F_EXIT_ARGS"), const("F_ENTRY_OUT"),
            const("F_BLOCKED_UPSTREAM")) == (A.F_PRIORITIZED, A.F_HAS_ARG, A.F_EXIT_ARGS, A.F_ENTRY_OUT,
                                             A.F_BLOCKED_UPSTREAM)
    assert (const("ARG_NULL"), const("ARG_SCALAR"), const("ARG_LIST"), const("MAX_ARGS")) == (
        A.ARG_NULL, A.ARG_SCALAR, A.ARG_LIST, A.MAX_ARGS)
    assert (const("PASS"), const("PASS_WAIT"), const("BLOCK_FLOW"), const("BLOCK_DEGRADE"), const("BLOCK_PARAM"),
            const("NO_CHECK"), const("BLOCK_UPSTREAM")) == (A.PASS, A.PASS_WAIT, A.BLOCK_FLOW, A.BLOCK_DEGRADE,
                                                            A.BLOCK_PARAM, A.NO_CHECK, A.BLOCK_UPSTREAM)
    assert const("REF_NONE") == A.REF_NONE


def test_service_file_names_the_builder():
    svc = os.path.join(ROOT, "java", "src", "main", "resources", "META-INF", "services",
                       "com.alibaba.csp.sentinel.slotchain.SlotChainBuilder")
    cls = [l.strip() for l in open(svc) if l.strip() and not l.startswith("#")]
    assert cls == ["com.alibaba.csp.sentinel.gpu.GpuSlotChainBuilder"]
    src = open(os.path.join(JAVA, "GpuSlotChainBuilder.java")).read()
    assert "class GpuSlotChainBuilder implements SlotChainBuilder" in src
    assert "new GpuDecisionSlot()" in src


def test_init_func_makes_the_builder_deterministic():
    # SlotChainProvider takes the first non-default builder ServiceLoader finds (core/slotchain/
    # SlotChainProvider.java:57-68) and the param extension registers HotParamSlotChainBuilder too: an InitFunc
    # (run from Env's static initialiser before any chain, core/init/InitExecutor.java:40-63) installs the GPU
    # builder into the provider's resolved field and fails loudly unless a built chain holds GpuDecisionSlot
    svc = os.path.join(ROOT, "java", "src", "main", "resources", "META-INF", "services",
                       "com.alibaba.csp.sentinel.init.InitFunc")
    cls = [l.strip() for l in open(svc) if l.strip() and not l.startswith("#")]
    assert cls == ["com.alibaba.csp.sentinel.gpu.GpuChainInit"]
    src = open(os.path.join(JAVA, "GpuChainInit.java")).read()
    assert "class GpuChainInit implements InitFunc" in src
    assert "@InitOrder(Integer.MIN_VALUE)" in src                     # before every other InitFunc
    assert 'getDeclaredField("builder")' in src                       # SlotChainProvider.builder
    ref = "/root/reference/sentinel-core/src/main/java/com/alibaba/csp/sentinel/slotchain/SlotChainProvider.java"
    if os.path.exists(ref):  # the field the InitFunc sets is the one newSlotChain() returns from
        txt = open(ref).read()
        assert "private static volatile SlotChainBuilder builder" in txt and "return builder.build();" in txt
    assert "instanceof GpuDecisionSlot" in src


def _code(text):
    text = re.sub(r'"(\\.|[^"\\])*"', '""', text)
    return re.sub(r"/\*.*?\*/|//[^\n]*", "", text, flags=re.S)


def test_init_failure_refuses_entries_instead_of_throwing():
    # InitExecutor.doInit catches an InitFunc's exception and stops running the later ones
    # (core/init/InitExecutor.java:51-62), so GpuChainInit must never throw; a failure poisons the decision slot,
    # which refuses entries with a BlockException (CtSph exits and rethrows those, core/CtSph.java:157-166)
    ref = "/root/reference/sentinel-core/src/main/java/com/alibaba/csp/sentinel/init/InitExecutor.java"
    if os.path.exists(ref):
        txt = open(ref).read()
        assert "w.func.init();" in txt and "catch (Exception ex)" in txt  # the loop is inside the catch
    init = _code(open(os.path.join(JAVA, "GpuChainInit.java")).read())
    assert "throw " not in init                                        # no exception reaches InitExecutor
    assert re.search(r"public void init\(\)\s*\{\s*try\s*\{\s*install\(\);\s*\}\s*catch \(Throwable", init)
    assert "failure = " in init and "public static String failure()" in init
    exc = _code(open(os.path.join(JAVA, "GpuUnavailableException.java")).read())
    assert "class GpuUnavailableException extends BlockException" in exc
    slot = _code(open(os.path.join(JAVA, "GpuDecisionSlot.java")).read())
    body = slot[slot.index("public void entry("):]
    body = body[:body.index("String name = resourceWrapper.getName();")]
    # the poison check is the first thing an entry does, and an engine that cannot be created poisons too
    assert re.search(r"GpuChainInit\.failure\(\);\s*if \(down != null\)\s*\{\s*throw new GpuUnavailableException", body)
    assert "GpuChainInit.fail(" in body and body.count("throw new GpuUnavailableException") == 2


def test_runtime_engine_failure_fails_closed():
    # once the engine dies at run time (a batch failed: e->fatal, BF_POOL_FULL, a poisoned
    # batcher) GpuEngine.decide throws a RuntimeException; CtSph.entryWithPriority catches anything that is not a
    # BlockException and lets the entry pass unchecked (core/CtSph.java:163-166).  The slot must record the failure
    # (every later entry refused by the poison check) and throw GpuUnavailableException (a BlockException)
    ref = "/root/reference/sentinel-core/src/main/java/com/alibaba/csp/sentinel/CtSph.java"
    if os.path.exists(ref):
        txt = open(ref).read()
        assert "catch (BlockException e1)" in txt and "catch (Throwable e1)" in txt
    slot = _code(open(os.path.join(JAVA, "GpuDecisionSlot.java")).read())
    body = slot[slot.index("public void entry("):slot.index("public void exit(")]
    m = re.search(r"try\s*\{\s*d = eng\.decide\(op\);\s*\}\s*catch \(RuntimeException (\w+)\)\s*\{(.*?)\}", body, re.S)
    assert m, "eng.decide is not guarded"
    handler = m.group(2)
    assert "GpuChainInit.fail(" in handler and "throw new GpuUnavailableException(GpuChainInit.failure())" in handler
    assert body.count("eng.decide(") == 1
    # GpuEngine.decide reports a dead engine with a RuntimeException (not an Error the guard would miss)
    eng = _code(open(os.path.join(JAVA, "GpuEngine.java")).read())
    dec = eng[eng.index("int decide(Op op)"):]
    assert "throw new IllegalStateException" in dec[:dec.index("\n    }")]


def test_java_sources_are_balanced():
    for root, _, files in os.walk(os.path.join(ROOT, "java", "src")):
        for f in files:
            if f.endswith(".java"):
                text = open(os.path.join(root, f)).read()
                text = re.sub(r'"(\\.|[^"\\])*"', '""', text)          # strings
                text = re.sub(r"'(\\.|[^'\\])'", "''", text)            # chars
                text = re.sub(r"/\*.*?\*/|//[^\n]*", "", text, flags=re.S)  # comments
                for a, b in ("{}", "()", "[]"):
                    assert text.count(a) == text.count(b), (f, a + b)
                pkg = re.search(r"^package ([\w.]+);", text, re.M).group(1)
                assert root.endswith(pkg.replace(".", os.sep)), (f, pkg)


def test_replay_export_matches_the_harness_format(tmp_path):
    from tools import jvm_replay as J  # noqa: E402
    J.export(5, str(tmp_path), n_entries=200, n_res=10, n_param_values=30)
    names = open(tmp_path / "resources.txt").read().splitlines()
    ev = np.fromfile(tmp_path / "events.bin", dtype=A.EVENT_DTYPE)
    assert len(names) == 10 and len(ev) == 400
    harness = open(os.path.join(ROOT, "java", "src", "test", "java", "com", "alibaba", "csp", "sentinel", "gpu",
                                "ReplayHarness.java")).read()
    # param.tsv: 16 fields, the harness reads f[0..10]
    for line in open(tmp_path / "param.tsv"):
        assert len(line.rstrip("\n").split("\t")) == 16
    assert "f[10].split" in harness
    # args.tsv: every HAS_ARG entry, with a value whose key is the event's aux
    rows = [l.rstrip("\n").split("\t") for l in open(tmp_path / "args.tsv")]
    assert len(rows) == int(((ev["kind"] == 0) & ((ev["flags"] & A.F_HAS_ARG) != 0)).sum())
    for idx, cls, text in rows[:50]:
        assert engine.param_key(text, cls) == int(ev["aux"][int(idx)])
