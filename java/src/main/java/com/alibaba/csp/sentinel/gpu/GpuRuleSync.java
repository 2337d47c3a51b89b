package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.lang.invoke.MethodHandle;
import java.lang.reflect.Field;
import java.util.ArrayList;
import java.util.Collections;
import java.util.HashMap;
import java.util.HashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

import com.alibaba.csp.sentinel.property.PropertyListener;
import com.alibaba.csp.sentinel.property.SentinelProperty;
import com.alibaba.csp.sentinel.slots.block.RuleConstant;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleManager;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRuleUtil;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.util.StringUtil;

import static java.lang.foreign.ValueLayout.JAVA_INT;

/**
 * Keeps the device rule tables equal to the three rule managers.  Each manager holds its rules in a
 * private {@code currentProperty} (FlowRuleManager.java:52, DegradeRuleManager.java:49,
 * ParamFlowRuleManager.java:45) that every loadRules / register2Property goes through; this class adds
 * one more {@link PropertyListener} to it, which pushes the new list through sg_load_*_rules (the engine
 * validates, de-duplicates and orders exactly as the managers do).  A register2Property swaps the
 * property object; {@link #rehook} (called by the batcher before every batch) follows the swap.
 *
 * <p>It also keeps, per resource, the rule lists in the engine's order, so that a decision word's
 * {@code rule_slot} names the very rule object the reference would put in its BlockException.
 */
final class GpuRuleSync {

    private static final Field[] FIELDS = new Field[3];
    private static final Object[] HOOKED = new Object[3];

    static volatile Map<String, List<FlowRule>> flowByResource = Collections.emptyMap();
    static volatile Map<String, List<DegradeRule>> degradeByResource = Collections.emptyMap();

    private static GpuEngine engine;

    private GpuRuleSync() {}

    static synchronized void attach(GpuEngine e) {
        engine = e;
        try {
            FIELDS[0] = FlowRuleManager.class.getDeclaredField("currentProperty");
            FIELDS[1] = DegradeRuleManager.class.getDeclaredField("currentProperty");
            FIELDS[2] = ParamFlowRuleManager.class.getDeclaredField("currentProperty");
            for (Field f : FIELDS) {
                f.setAccessible(true);
            }
        } catch (ReflectiveOperationException ex) {
            throw new IllegalStateException("sentinel_gpu: rule managers without currentProperty", ex);
        }
        rehook();
    }

    /** Hook any manager whose property object changed since the last call (cheap when none did). */
    @SuppressWarnings("unchecked")
    static void rehook() {
        for (int k = 0; k < 3; k++) {
            Object p;
            try {
                p = FIELDS[k].get(null);
            } catch (IllegalAccessException ex) {
                throw new IllegalStateException(ex);
            }
            if (p == HOOKED[k]) {
                continue;
            }
            synchronized (GpuRuleSync.class) {
                if (p == HOOKED[k]) {
                    continue;
                }
                HOOKED[k] = p;
                switch (k) {
                    case 0:
                        ((SentinelProperty<List<FlowRule>>)p).addListener(new Listener<>(GpuRuleSync::loadFlow));
                        break;
                    case 1:
                        ((SentinelProperty<List<DegradeRule>>)p).addListener(
                            new Listener<>(GpuRuleSync::loadDegrade));
                        break;
                    default:
                        ((SentinelProperty<List<ParamFlowRule>>)p).addListener(new Listener<>(GpuRuleSync::loadParam));
                }
            }
        }
    }

    private interface Loader<T> {
        void load(List<T> rules);
    }

    private static final class Listener<T> implements PropertyListener<List<T>> {
        private final Loader<T> loader;

        Listener(Loader<T> loader) {
            this.loader = loader;
        }

        @Override
        public void configUpdate(List<T> value) {
            loader.load(value == null ? Collections.<T>emptyList() : value);
        }

        @Override
        public void configLoad(List<T> value) {
            loader.load(value == null ? Collections.<T>emptyList() : value);
        }
    }

    private static void push(MethodHandle fn, MemorySegment rules, int n, String what) {
        synchronized (engine.nativeLock) {
            try (Arena a = Arena.ofConfined()) {
                MemorySegment kept = a.allocate(JAVA_INT);
                SentinelGpu.check((int)fn.invokeExact(engine.handle, rules, n, kept));
            } catch (RuntimeException ex) {
                throw ex;
            } catch (Throwable t) {
                throw new IllegalStateException("sentinel_gpu: loading " + what + " rules failed", t);
            }
        }
    }

    static void loadFlow(List<FlowRule> rules) {
        try (Arena a = Arena.ofConfined()) {
            push(SentinelGpu.LOAD_FLOW_RULES, NativeRules.flow(a, rules), rules.size(), "flow");
        }
        // FlowRuleManager's own grouping and FlowRuleComparator order (FlowRuleUtil.java:89-158)
        flowByResource = FlowRuleUtil.buildFlowRuleMap(rules);
    }

    static void loadDegrade(List<DegradeRule> rules) {
        try (Arena a = Arena.ofConfined()) {
            push(SentinelGpu.LOAD_DEGRADE_RULES, NativeRules.degrade(a, rules), rules.size(), "degrade");
        }
        // DegradeRuleManager.loadDegradeConf (DegradeRuleManager.java:177-205): a HashSet per resource
        Map<String, Set<DegradeRule>> sets = new HashMap<>();
        for (DegradeRule r : rules) {
            if (!DegradeRuleManager.isValidRule(r)) {
                continue;
            }
            if (StringUtil.isBlank(r.getLimitApp())) {
                r.setLimitApp(RuleConstant.LIMIT_APP_DEFAULT);
            }
            sets.computeIfAbsent(r.getResource(), k -> new HashSet<>()).add(r);
        }
        Map<String, List<DegradeRule>> lists = new HashMap<>();
        for (Map.Entry<String, Set<DegradeRule>> en : sets.entrySet()) {
            lists.put(en.getKey(), new ArrayList<>(en.getValue()));
        }
        degradeByResource = lists;
    }

    static void loadParam(List<ParamFlowRule> rules) {
        try (Arena a = Arena.ofConfined()) {
            push(SentinelGpu.LOAD_PARAM_RULES, NativeRules.param(a, rules), rules.size(), "param");
        }
        // the rule objects of a block come from ParamFlowRuleManager.getRulesOfResource, same order
    }

    static FlowRule flowRule(String resource, int slot) {
        List<FlowRule> l = flowByResource.get(resource);
        return l != null && slot < l.size() ? l.get(slot) : null;
    }

    static DegradeRule degradeRule(String resource, int slot) {
        List<DegradeRule> l = degradeByResource.get(resource);
        return l != null && slot < l.size() ? l.get(slot) : null;
    }

    static ParamFlowRule paramRule(String resource, int slot) {
        List<ParamFlowRule> l = ParamFlowRuleManager.getRulesOfResource(resource);
        return l != null && slot < l.size() ? l.get(slot) : null;
    }
}
