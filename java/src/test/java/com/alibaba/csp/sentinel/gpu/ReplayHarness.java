package com.alibaba.csp.sentinel.gpu;

import java.io.BufferedWriter;
import java.io.IOException;
import java.lang.reflect.Field;
import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.charset.StandardCharsets;
import java.nio.file.Files;
import java.nio.file.Path;
import java.nio.file.Paths;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;
import java.util.TreeSet;
import java.util.concurrent.atomic.AtomicReferenceArray;

import com.alibaba.csp.sentinel.AsyncEntry;
import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.SphU;
import com.alibaba.csp.sentinel.Tracer;
import com.alibaba.csp.sentinel.node.ClusterNode;
import com.alibaba.csp.sentinel.node.StatisticNode;
import com.alibaba.csp.sentinel.slots.block.AbstractRule;
import com.alibaba.csp.sentinel.slots.block.BlockException;
import com.alibaba.csp.sentinel.slots.block.RuleConstant;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeException;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleUtil;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowItem;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.slots.clusterbuilder.ClusterBuilderSlot;
import com.alibaba.csp.sentinel.slots.statistic.MetricEvent;
import com.alibaba.csp.sentinel.slots.statistic.base.LeapArray;
import com.alibaba.csp.sentinel.slots.statistic.base.WindowWrap;
import com.alibaba.csp.sentinel.slots.statistic.data.MetricBucket;
import com.alibaba.csp.sentinel.slots.statistic.metric.ArrayMetric;
import com.alibaba.csp.sentinel.util.StringUtil;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * Replays an exported trace (tools/jvm_replay.py export) through the UNMODIFIED reference slot chain
 * and writes what it decided, in the format tools/jvm_replay.py import turns into a tests/golden
 * fixture.  Every ENTRY is an AsyncEntry (SphU.asyncEntry, core/SphU.java:243) so that the trace's
 * interleaved exits need no nesting; the clock is the test-scope TimeUtil, set to each event's ts.
 *
 * <p>Decision words: status | rule_slot << 8, the rule's index in the manager's per-resource list
 * (FlowRuleUtil.buildFlowRuleMap order; the DegradeRuleManager HashSet; getRulesOfResource), which is
 * how sentinel_gpu.h numbers rule slots.  Waits stay 0: a RateLimiter wait is a real sleep inside the
 * reference and is not reported.
 *
 * <p>Usage: {@code ReplayHarness IN_DIR OUT_DIR}.
 */
public final class ReplayHarness {

    private static final String NULL = "\\N";
    private static final int EV_ENTRY = 0, EV_EXIT = 1, EV_TRACE = 2;
    private static final int F_EXIT_ARGS = 4;
    private static final long REF_MASK = 0xFFFFFFFFFFFFL;

    private ReplayHarness() {}

    private static String str(String s) {
        return NULL.equals(s) ? null : s;
    }

    private static List<String[]> rows(Path p) throws IOException {
        List<String[]> out = new ArrayList<>();
        if (!Files.exists(p)) {
            return out;
        }
        for (String line : Files.readAllLines(p, StandardCharsets.UTF_8)) {
            if (!line.isEmpty()) {
                out.add(line.split("\t", -1));
            }
        }
        return out;
    }

    static List<FlowRule> flowRules(Path p) throws IOException {
        List<FlowRule> rules = new ArrayList<>();
        for (String[] f : rows(p)) {
            FlowRule r = new FlowRule();
            r.setResource(str(f[0]));
            r.setLimitApp(str(f[1]));
            r.setRefResource(str(f[2]));
            r.setCount(Double.parseDouble(f[3]));
            r.setGrade(Integer.parseInt(f[4]));
            r.setStrategy(Integer.parseInt(f[5]));
            r.setControlBehavior(Integer.parseInt(f[6]));
            r.setWarmUpPeriodSec(Integer.parseInt(f[7]));
            r.setMaxQueueingTimeMs(Integer.parseInt(f[8]));
            r.setClusterMode(Integer.parseInt(f[9]) != 0);
            // cluster fields f[10..15]: cluster rules need a token client, which a replay has not
            rules.add(r);
        }
        return rules;
    }

    static List<DegradeRule> degradeRules(Path p) throws IOException {
        List<DegradeRule> rules = new ArrayList<>();
        for (String[] f : rows(p)) {
            DegradeRule r = new DegradeRule(str(f[0]));
            r.setLimitApp(str(f[1]));
            r.setCount(Double.parseDouble(f[2]));
            r.setTimeWindow(Integer.parseInt(f[3]));
            r.setGrade(Integer.parseInt(f[4]));
            rules.add(r);
        }
        return rules;
    }

    static List<ParamFlowRule> paramRules(Path p) throws IOException {
        List<ParamFlowRule> rules = new ArrayList<>();
        for (String[] f : rows(p)) {
            ParamFlowRule r = new ParamFlowRule(str(f[0]));
            r.setLimitApp(str(f[1]));
            r.setCount(Double.parseDouble(f[2]));
            r.setDurationInSec(Long.parseLong(f[3]));
            r.setGrade(Integer.parseInt(f[4]));
            r.setParamIdx(NULL.equals(f[5]) ? null : Integer.valueOf(f[5]));
            r.setControlBehavior(Integer.parseInt(f[6]));
            r.setMaxQueueingTimeMs(Integer.parseInt(f[7]));
            r.setBurstCount(Integer.parseInt(f[8]));
            r.setClusterMode(Integer.parseInt(f[9]) != 0);
            List<ParamFlowItem> items = new ArrayList<>();
            if (!NULL.equals(f[10])) {
                for (String it : f[10].split("\u001e", -1)) {
                    String[] g = it.split("\u001f", -1);
                    ParamFlowItem item = new ParamFlowItem();
                    item.setObject(str(g[0]));
                    item.setClassType(str(g[1]));
                    item.setCount(NULL.equals(g[2]) ? null : Integer.valueOf(g[2]));
                    items.add(item);
                }
            }
            r.setParamFlowItemList(items);
            rules.add(r);
        }
        return rules;
    }

    static Object argValue(String cls, String text) {
        switch (cls) {
            case "java.lang.Integer":
                return Integer.valueOf(text);
            case "java.lang.Long":
                return Long.valueOf(text);
            case "java.lang.Byte":
                return Byte.valueOf(text);
            case "java.lang.Short":
                return Short.valueOf(text);
            case "java.lang.Boolean":
                return Boolean.valueOf(text);
            default:
                return text;
        }
    }

    private static int indexOf(List<? extends AbstractRule> list, AbstractRule r) {
        if (list == null) {
            return 0;
        }
        for (int i = 0; i < list.size(); i++) {
            if (list.get(i) == r) {
                return i;
            }
        }
        int k = list.indexOf(r);
        return k < 0 ? 0 : k;
    }

    public static void main(String[] argv) throws Exception {
        Path in = Paths.get(argv[0]);
        Path out = Paths.get(argv[1]);
        Files.createDirectories(out);
        List<String> names = Files.readAllLines(in.resolve("resources.txt"), StandardCharsets.UTF_8);

        List<FlowRule> flow = flowRules(in.resolve("flow.tsv"));
        List<DegradeRule> degrade = degradeRules(in.resolve("degrade.tsv"));
        List<ParamFlowRule> param = paramRules(in.resolve("param.tsv"));
        FlowRuleManager.loadRules(flow);
        DegradeRuleManager.loadRules(degrade);
        ParamFlowRuleManager.loadRules(param);
        Map<String, List<FlowRule>> flowByRes = FlowRuleUtil.buildFlowRuleMap(flow);
        Map<String, List<DegradeRule>> degByRes = new HashMap<>();
        Map<String, Set<DegradeRule>> sets = new HashMap<>();
        for (DegradeRule r : degrade) {
            if (DegradeRuleManager.isValidRule(r)) {
                if (StringUtil.isBlank(r.getLimitApp())) {
                    r.setLimitApp(RuleConstant.LIMIT_APP_DEFAULT);
                }
                sets.computeIfAbsent(r.getResource(), k -> new HashSet<>()).add(r);
            }
        }
        for (Map.Entry<String, Set<DegradeRule>> e : sets.entrySet()) {
            degByRes.put(e.getKey(), new ArrayList<>(e.getValue()));
        }

        Map<Integer, Object> args = new HashMap<>();
        for (String[] f : rows(in.resolve("args.tsv"))) {
            args.put(Integer.valueOf(f[0]), argValue(f[1], f[2]));
        }

        byte[] raw = Files.readAllBytes(in.resolve("events.bin"));
        ByteBuffer bb = ByteBuffer.wrap(raw).order(ByteOrder.LITTLE_ENDIAN);
        int n = raw.length / 24;
        AsyncEntry[] entries = new AsyncEntry[n];
        Object[][] entryArgs = new Object[n][];
        ByteBuffer dec = ByteBuffer.allocate(4 * n).order(ByteOrder.LITTLE_ENDIAN);
        Set<Integer> touched = new TreeSet<>();
        for (int i = 0; i < n; i++) {
            long ts = bb.getLong(24 * i);
            int res = bb.getInt(24 * i + 8);
            int count = bb.getShort(24 * i + 12) & 0xFFFF;
            int kind = bb.get(24 * i + 14);
            int flags = bb.get(24 * i + 15) & 0xFF;
            long aux = bb.getLong(24 * i + 16);
            String name = names.get(res);
            touched.add(res);
            TimeUtil.set(ts);
            int word = 0xFF;
            if (kind == EV_ENTRY) {
                Object[] a = args.containsKey(i) ? new Object[] {args.get(i)} : new Object[0];
                entryArgs[i] = a;
                try {
                    entries[i] = SphU.asyncEntry(name, EntryType.IN, count, a);
                    word = 0;
                } catch (BlockException be) {
                    if (be instanceof FlowException) {
                        word = 2 | indexOf(flowByRes.get(name), be.getRule()) << 8;
                    } else if (be instanceof DegradeException) {
                        word = 3 | indexOf(degByRes.get(name), be.getRule()) << 8;
                    } else if (be instanceof ParamFlowException) {
                        word = 4 | indexOf(ParamFlowRuleManager.getRulesOfResource(name),
                                           ((ParamFlowException)be).getRule()) << 8;
                    } else {
                        word = 6;
                    }
                }
            } else {
                int ref = (int)(aux & REF_MASK);
                AsyncEntry e = ref < n ? entries[ref] : null;
                if (e != null && kind == EV_EXIT) {
                    if ((flags & F_EXIT_ARGS) != 0) {
                        e.exit(count, entryArgs[ref]);
                    } else {
                        e.exit(count);
                    }
                    entries[ref] = null;
                } else if (e != null && kind == EV_TRACE) {
                    Tracer.traceEntry(new RuntimeException("replayed trace"), count, e);
                }
            }
            dec.putInt(4 * i, word);
        }
        Files.write(out.resolve("decisions.bin"), dec.array());

        try (BufferedWriter w = Files.newBufferedWriter(out.resolve("nodes.tsv"), StandardCharsets.UTF_8)) {
            for (int res : touched) {
                ClusterNode cn = ClusterBuilderSlot.getClusterNode(names.get(res));
                if (cn == null) {
                    continue;
                }
                dump(w, res, "s", buckets(cn, "rollingCounterInSecond"));
                dump(w, res, "m", buckets(cn, "rollingCounterInMinute"));
            }
        }
        System.out.println("replayed " + n + " events");
    }

    @SuppressWarnings("unchecked")
    private static AtomicReferenceArray<WindowWrap<MetricBucket>> buckets(ClusterNode cn, String field)
        throws ReflectiveOperationException {
        Field f = StatisticNode.class.getDeclaredField(field);
        f.setAccessible(true);
        ArrayMetric m = (ArrayMetric)f.get(cn);
        Field d = ArrayMetric.class.getDeclaredField("data");
        d.setAccessible(true);
        LeapArray<MetricBucket> la = (LeapArray<MetricBucket>)d.get(m);
        Field a = LeapArray.class.getDeclaredField("array");
        a.setAccessible(true);
        return (AtomicReferenceArray<WindowWrap<MetricBucket>>)a.get(la);
    }

    private static void dump(BufferedWriter w, int res, String which, AtomicReferenceArray<WindowWrap<MetricBucket>> arr)
        throws IOException {
        for (int s = 0; s < arr.length(); s++) {
            WindowWrap<MetricBucket> ww = arr.get(s);
            if (ww == null) {
                continue;
            }
            MetricBucket b = ww.value();
            w.write(res + "\t" + which + "\t" + s + "\t" + ww.windowStart() + "\t" + b.get(MetricEvent.PASS) + "\t"
                    + b.get(MetricEvent.BLOCK) + "\t" + b.get(MetricEvent.EXCEPTION) + "\t"
                    + b.get(MetricEvent.SUCCESS) + "\t" + b.get(MetricEvent.RT) + "\t"
                    + b.get(MetricEvent.OCCUPIED_PASS) + "\t" + b.minRt() + "\n");
        }
    }
}
