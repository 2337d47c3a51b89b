package com.alibaba.csp.sentinel.gpu;

import java.util.concurrent.ConcurrentHashMap;

import com.alibaba.csp.sentinel.Constants;
import com.alibaba.csp.sentinel.Entry;
import com.alibaba.csp.sentinel.EntryType;
import com.alibaba.csp.sentinel.context.Context;
import com.alibaba.csp.sentinel.node.DefaultNode;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotEntryCallback;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotExitCallback;
import com.alibaba.csp.sentinel.slotchain.ResourceWrapper;
import com.alibaba.csp.sentinel.slots.block.BlockException;
import com.alibaba.csp.sentinel.slots.block.authority.AuthoritySlot;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeException;
import com.alibaba.csp.sentinel.slots.block.degrade.DegradeRule;
import com.alibaba.csp.sentinel.slots.block.flow.FlowException;
import com.alibaba.csp.sentinel.slots.block.flow.FlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowException;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRule;
import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowRuleManager;
import com.alibaba.csp.sentinel.slots.statistic.StatisticSlotCallbackRegistry;
import com.alibaba.csp.sentinel.slots.system.SystemSlot;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * The GPU-decided part of HotParamSlotChainBuilder's chain (param/slots/HotParamSlotChainBuilder.java:38-51):
 * StatisticSlot -> ParamFlowSlot -> SystemSlot -> AuthoritySlot -> FlowSlot -> DegradeSlot in one slot.
 *
 * <p>SystemSlot and AuthoritySlot stay on the JVM (their inputs -- system load, the origin's black/white
 * list -- live here) and run first; a BlockException of theirs is passed to the engine as
 * SG_F_BLOCKED_UPSTREAM, so the param checks that precede them in the reference still run and may block
 * first.  The engine decides everything else and keeps the resource, origin and context statistics
 * (StatisticSlot.entry/exit, StatisticSlot.java:54-173) on the device; the JVM keeps
 * {@link Constants#ENTRY_NODE} and the registered entry/exit callbacks, minus the hot-parameter ones
 * whose thread counts the engine keeps itself.
 */
public class GpuDecisionSlot extends AbstractLinkedProcessorSlot<DefaultNode> {

    private static final String PARAM_PKG = "com.alibaba.csp.sentinel.slots.block.flow.param.";

    private final SystemSlot system = new SystemSlot();
    private final AuthoritySlot authority = new AuthoritySlot();
    /** Passed entries of every chain (one slot instance per resource) awaiting their exit. */
    private static final ConcurrentHashMap<Entry, GpuEngine.Op> LIVE = new ConcurrentHashMap<>();

    @Override
    public void entry(Context context, ResourceWrapper resourceWrapper, DefaultNode node, int count,
                      boolean prioritized, Object... args) throws Throwable {
        // fail closed and visibly: a drop-in that could not take over the path refuses the entry (a
        // BlockException the caller sees) rather than pass it with no rule checked
        String down = GpuChainInit.failure();
        if (down != null) {
            throw new GpuUnavailableException(down);
        }
        GpuEngine eng;
        try {
            eng = GpuEngine.get();
        } catch (RuntimeException ex) {
            GpuChainInit.fail("engine creation failed", ex);
            throw new GpuUnavailableException(GpuChainInit.failure());
        }
        String name = resourceWrapper.getName();
        if (count < 0 || count > 0xFFFF) {
            throw new IllegalArgumentException("sentinel_gpu: acquire count " + count + " outside [0, 65535]");
        }
        BlockException upstream = null;
        try {
            system.entry(context, resourceWrapper, node, count, prioritized, args);    // no next slot: checks only
            authority.entry(context, resourceWrapper, node, count, prioritized, args);
        } catch (BlockException be) {
            upstream = be;
        }
        boolean hasParam = args != null && ParamFlowRuleManager.hasRules(name);
        if (hasParam) {
            if (args.length > SentinelGpu.MAX_ARGS) {
                throw new IllegalArgumentException("sentinel_gpu: more than " + SentinelGpu.MAX_ARGS
                                                   + " arguments on a resource with hot-parameter rules");
            }
            // ParamFlowSlot.applyRealParamIdx mutates the rule beans (ParamFlowSlot.java:65-75); the engine
            // resolves the same index on the device, the beans are kept in step for getRules() readers
            for (ParamFlowRule r : ParamFlowRuleManager.getRulesOfResource(name)) {
                int idx = r.getParamIdx();
                if (idx < 0) {
                    r.setParamIdx(-idx <= args.length ? args.length + idx : -idx);
                }
            }
        }
        int flags = (prioritized ? SentinelGpu.F_PRIORITIZED : 0)
            | (resourceWrapper.getType() == EntryType.OUT ? SentinelGpu.F_ENTRY_OUT : 0)
            | (upstream != null ? SentinelGpu.F_BLOCKED_UPSTREAM : 0);
        GpuEngine.Op op = new GpuEngine.Op(TimeUtil.currentTimeMillis(), eng.resourceId(name), count,
                                           SentinelGpu.EV_ENTRY, flags, 0L, eng.originId(context.getOrigin()),
                                           eng.contextId(context.getName()), hasParam ? args : null,
                                           Thread.currentThread());
        int d;
        try {
            d = eng.decide(op);
        } catch (RuntimeException ex) {
            // the engine died at run time (a batch failed: a full map pool, a poisoned batcher, a device error).
            // CtSph.entryWithPriority catches anything but a BlockException and lets the entry pass unchecked
            // (core/CtSph.java:163-166), so record the failure and fail closed, for this entry and every later one
            GpuChainInit.fail("the engine failed at run time", ex);
            throw new GpuUnavailableException(GpuChainInit.failure());
        }
        int status = SentinelGpu.status(d);
        boolean in = resourceWrapper.getType() == EntryType.IN;
        switch (status) {
            case SentinelGpu.PASS:
            case SentinelGpu.PASS_WAIT: {
                int wait = SentinelGpu.waitMs(d);
                if (wait > 0) {
                    Thread.sleep(wait);   // RateLimiterController / DefaultController.canPass sleep in the caller
                }
                LIVE.put(context.getCurEntry(), op);
                if (in) {
                    Constants.ENTRY_NODE.increaseThreadNum();
                    if (status == SentinelGpu.PASS) {
                        Constants.ENTRY_NODE.addPassRequest(count);
                    }
                }
                for (ProcessorSlotEntryCallback<DefaultNode> h : StatisticSlotCallbackRegistry.getEntryCallbacks()) {
                    if (!h.getClass().getName().startsWith(PARAM_PKG)) {
                        h.onPass(context, resourceWrapper, node, count, args);
                    }
                }
                fireEntry(context, resourceWrapper, node, count, prioritized, args);
                return;
            }
            case SentinelGpu.NO_CHECK:
                fireEntry(context, resourceWrapper, node, count, prioritized, args);
                return;
            default:
                break;
        }
        BlockException e = blockOf(status, SentinelGpu.ruleSlot(d), name, args, upstream);
        context.getCurEntry().setError(e);
        if (in) {
            Constants.ENTRY_NODE.increaseBlockQps(count);
        }
        for (ProcessorSlotEntryCallback<DefaultNode> h : StatisticSlotCallbackRegistry.getEntryCallbacks()) {
            if (!h.getClass().getName().startsWith(PARAM_PKG)) {
                h.onBlocked(e, context, resourceWrapper, node, count, args);
            }
        }
        throw e;
    }

    private static BlockException blockOf(int status, int slot, String name, Object[] args, BlockException upstream) {
        switch (status) {
            case SentinelGpu.BLOCK_FLOW: {
                FlowRule r = GpuRuleSync.flowRule(name, slot);
                return new FlowException(r == null ? null : r.getLimitApp(), r);
            }
            case SentinelGpu.BLOCK_DEGRADE: {
                DegradeRule r = GpuRuleSync.degradeRule(name, slot);
                return new DegradeException(r == null ? null : r.getLimitApp(), r);
            }
            case SentinelGpu.BLOCK_PARAM: {
                ParamFlowRule r = GpuRuleSync.paramRule(name, slot);
                String triggered = "";
                if (r != null && args != null && r.getParamIdx() >= 0 && args.length > r.getParamIdx()) {
                    triggered = String.valueOf(args[r.getParamIdx()]);
                }
                return new ParamFlowException(name, triggered, r);
            }
            case SentinelGpu.BLOCK_UPSTREAM:
                if (upstream != null) {
                    return upstream;
                }
                // fall through: the engine never reports this without the flag
            default:
                throw new IllegalStateException("sentinel_gpu: unexpected decision status " + status);
        }
    }

    @Override
    public void exit(Context context, ResourceWrapper resourceWrapper, int count, Object... args) {
        Entry cur = context.getCurEntry();
        GpuEngine.Op entry = LIVE.remove(cur);
        if (entry != null && cur.getError() == null) {
            GpuEngine eng = GpuEngine.get();
            long now = TimeUtil.currentTimeMillis();
            long rtRaw = now - cur.getCreateTime();
            boolean withArgs = args != null && args.length > 0 && ParamFlowRuleManager.hasRules(resourceWrapper.getName());
            eng.post(new GpuEngine.Op(now, entry.resId, count, SentinelGpu.EV_EXIT,
                                      withArgs ? SentinelGpu.F_EXIT_ARGS : 0,
                                      SentinelGpu.auxExit(GpuEngine.indexOf(entry), rtRaw), entry.origin,
                                      entry.context, withArgs ? args : null, null));
            if (resourceWrapper.getType() == EntryType.IN) {
                Constants.ENTRY_NODE.addRtAndSuccess(Math.min(rtRaw, Constants.TIME_DROP_VALVE), count);
                Constants.ENTRY_NODE.decreaseThreadNum();
            }
        }
        for (ProcessorSlotExitCallback h : StatisticSlotCallbackRegistry.getExitCallbacks()) {
            if (!h.getClass().getName().startsWith(PARAM_PKG)) {
                h.onExit(context, resourceWrapper, count, args);
            }
        }
        fireExit(context, resourceWrapper, count, args);
    }

    /** Tracer.trace(t, count) for an entry of this chain (core/Tracer.java:47-59 -> ClusterNode.trace). */
    static void trace(Entry cur, int count) {
        GpuEngine.Op entry = LIVE.get(cur);
        if (entry != null) {
            GpuEngine.get().post(new GpuEngine.Op(TimeUtil.currentTimeMillis(), entry.resId, count,
                                                  SentinelGpu.EV_TRACE, 0,
                                                  SentinelGpu.auxExit(GpuEngine.indexOf(entry), 0), entry.origin,
                                                  entry.context, null, null));
        }
    }
}
