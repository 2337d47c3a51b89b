package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.Entry;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.context.ContextUtil;
import com.alibaba.csp.sentinel.slots.block.BlockException;

/**
 * Tracer for entries decided by {@link GpuDecisionSlot}: the exception counters of the resource live on
 * the device, so {@code Tracer.trace(t, count)} (core/Tracer.java:47-59), which adds to the JVM-side
 * ClusterNode, becomes a TRACE event.  Same filtering as the reference: null and BlockException are
 * ignored, and so is a call outside any entry.
 */
public final class GpuTracer {

    private GpuTracer() {}

    public static void trace(Throwable e) {
        trace(e, 1);
    }

    public static void trace(Throwable e, int count) {
        if (e == null || e instanceof BlockException) {
            return;
        }
        traceContext(e, count, ContextUtil.getContext());
    }

    /** Tracer.traceContext(Throwable, int, Context) */
    public static void traceContext(Throwable e, int count, Context context) {
        if (context == null || context.getCurEntry() == null) {
            return;
        }
        traceEntry(e, count, context.getCurEntry());
    }

    /** Tracer.traceEntry(Throwable, int, Entry) */
    public static void traceEntry(Throwable e, int count, Entry entry) {
        if (e == null || e instanceof BlockException || entry == null) {
            return;
        }
        GpuDecisionSlot.trace(entry, count);
    }
}
