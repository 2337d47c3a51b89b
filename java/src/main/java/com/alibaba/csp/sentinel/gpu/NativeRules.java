package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;
import java.util.List;

import com.alibaba.csp.sentinel.slots.block.ClusterRuleConstant;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.flow.ClusterFlowConfig;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowClusterConfig;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowItem;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * The rule beans as the C structs of sentinel_gpu.h (sg_flow_rule, sg_degrade_rule, sg_param_rule,
 * sg_param_item): field for field, with the beans' own defaults, strings as UTF-8 in the caller's arena.
 * Offsets are those of SentinelGpu's layouts (checked against the C compiler by the tests).
 */
final class NativeRules {

    private NativeRules() {}

    private static MemorySegment str(Arena a, String s) {
        return s == null ? MemorySegment.NULL : a.allocateFrom(s);
    }

    private static long off(java.lang.foreign.StructLayout l, String field) {
        return l.byteOffset(java.lang.foreign.MemoryLayout.PathElement.groupElement(field));
    }

    /** FlowRule (core/slots/block/flow/FlowRule.java:40-90) + ClusterFlowConfig -> sg_flow_rule[] */
    static MemorySegment flow(Arena a, List<FlowRule> rules) {
        final java.lang.foreign.StructLayout L = SentinelGpu.SG_FLOW_RULE;
        MemorySegment m = a.allocate(L, Math.max(1, rules.size()));
        for (int i = 0; i < rules.size(); i++) {
            FlowRule r = rules.get(i);
            MemorySegment s = m.asSlice(i * L.byteSize(), L.byteSize());
            s.set(ADDRESS, off(L, "resource"), str(a, r.getResource()));
            s.set(ADDRESS, off(L, "limit_app"), str(a, r.getLimitApp()));
            s.set(ADDRESS, off(L, "ref_resource"), str(a, r.getRefResource()));
            s.set(JAVA_DOUBLE, off(L, "count"), r.getCount());
            s.set(JAVA_INT, off(L, "grade"), r.getGrade());
            s.set(JAVA_INT, off(L, "strategy"), r.getStrategy());
            s.set(JAVA_INT, off(L, "control_behavior"), r.getControlBehavior());
            s.set(JAVA_INT, off(L, "warm_up_period_sec"), r.getWarmUpPeriodSec());
            s.set(JAVA_INT, off(L, "max_queueing_time_ms"), r.getMaxQueueingTimeMs());
            s.set(JAVA_INT, off(L, "cluster_mode"), r.isClusterMode() ? 1 : 0);
            ClusterFlowConfig c = r.getClusterConfig();
            s.set(JAVA_LONG, off(L, "cluster_flow_id"), c == null || c.getFlowId() == null ? 0L : c.getFlowId());
            s.set(JAVA_INT, off(L, "cluster_threshold_type"),
                  c == null ? ClusterRuleConstant.FLOW_THRESHOLD_AVG_LOCAL : c.getThresholdType());
            s.set(JAVA_INT, off(L, "cluster_fallback_to_local"), c == null || c.isFallbackToLocalWhenFail() ? 1 : 0);
            s.set(JAVA_INT, off(L, "cluster_strategy"), c == null ? 0 : c.getStrategy());
            s.set(JAVA_INT, off(L, "cluster_sample_count"), c == null ? 10 : c.getSampleCount());
            s.set(JAVA_INT, off(L, "cluster_window_interval_ms"), c == null ? 1000 : c.getWindowIntervalMs());
        }
        return m;
    }

    /** DegradeRule (core/slots/block/degrade/DegradeRule.java:60-140) -> sg_degrade_rule[] */
    static MemorySegment degrade(Arena a, List<DegradeRule> rules) {
        final java.lang.foreign.StructLayout L = SentinelGpu.SG_DEGRADE_RULE;
        MemorySegment m = a.allocate(L, Math.max(1, rules.size()));
        for (int i = 0; i < rules.size(); i++) {
            DegradeRule r = rules.get(i);
            MemorySegment s = m.asSlice(i * L.byteSize(), L.byteSize());
            s.set(ADDRESS, off(L, "resource"), str(a, r.getResource()));
            s.set(ADDRESS, off(L, "limit_app"), str(a, r.getLimitApp()));
            s.set(JAVA_DOUBLE, off(L, "count"), r.getCount());
            s.set(JAVA_INT, off(L, "time_window"), r.getTimeWindow());
            s.set(JAVA_INT, off(L, "grade"), r.getGrade());
        }
        return m;
    }

    /** ParamFlowRule (param/slots/block/flow/param/ParamFlowRule.java:40-70) -> sg_param_rule[] */
    static MemorySegment param(Arena a, List<ParamFlowRule> rules) {
        final java.lang.foreign.StructLayout L = SentinelGpu.SG_PARAM_RULE;
        final java.lang.foreign.StructLayout I = SentinelGpu.SG_PARAM_ITEM;
        MemorySegment m = a.allocate(L, Math.max(1, rules.size()));
        for (int i = 0; i < rules.size(); i++) {
            ParamFlowRule r = rules.get(i);
            MemorySegment s = m.asSlice(i * L.byteSize(), L.byteSize());
            s.set(ADDRESS, off(L, "resource"), str(a, r.getResource()));
            s.set(ADDRESS, off(L, "limit_app"), str(a, r.getLimitApp()));
            s.set(JAVA_DOUBLE, off(L, "count"), r.getCount());
            s.set(JAVA_LONG, off(L, "duration_in_sec"), r.getDurationInSec());
            s.set(JAVA_INT, off(L, "grade"), r.getGrade());
            s.set(JAVA_INT, off(L, "param_idx"), r.getParamIdx() == null ? 0 : r.getParamIdx());
            s.set(JAVA_INT, off(L, "has_param_idx"), r.getParamIdx() == null ? 0 : 1);
            s.set(JAVA_INT, off(L, "control_behavior"), r.getControlBehavior());
            s.set(JAVA_INT, off(L, "max_queueing_time_ms"), r.getMaxQueueingTimeMs());
            s.set(JAVA_INT, off(L, "burst_count"), r.getBurstCount());
            s.set(JAVA_INT, off(L, "cluster_mode"), r.isClusterMode() ? 1 : 0);
            List<ParamFlowItem> items = r.getParamFlowItemList();
            int n = items == null ? 0 : items.size();
            s.set(JAVA_INT, off(L, "n_items"), n);
            MemorySegment im = a.allocate(I, Math.max(1, n));
            for (int k = 0; k < n; k++) {
                ParamFlowItem it = items.get(k);
                MemorySegment t = im.asSlice(k * I.byteSize(), I.byteSize());
                t.set(ADDRESS, off(I, "object"), str(a, it.getObject()));
                t.set(ADDRESS, off(I, "class_type"), str(a, it.getClassType()));
                t.set(JAVA_INT, off(I, "count"), it.getCount() == null ? 0 : it.getCount());
                t.set(JAVA_INT, off(I, "has_count"), it.getCount() == null ? 0 : 1);
            }
            s.set(ADDRESS, off(L, "items"), im);
            ParamFlowClusterConfig c = r.getClusterConfig();
            s.set(JAVA_LONG, off(L, "cluster_flow_id"), c == null || c.getFlowId() == null ? 0L : c.getFlowId());
            s.set(JAVA_INT, off(L, "cluster_threshold_type"), c == null ? 0 : c.getThresholdType());
            s.set(JAVA_INT, off(L, "cluster_fallback_to_local"), c != null && c.isFallbackToLocalWhenFail() ? 1 : 0);
            s.set(JAVA_INT, off(L, "cluster_sample_count"), c == null ? 10 : c.getSampleCount());
            s.set(JAVA_INT, off(L, "cluster_window_interval_ms"), c == null ? 1000 : c.getWindowIntervalMs());
        }
        return m;
    }
}
