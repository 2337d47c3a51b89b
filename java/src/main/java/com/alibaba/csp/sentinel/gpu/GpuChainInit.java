package com.alibaba.csp.sentinel.gpu;

import java.lang.reflect.Field;

import com.alibaba.csp.sentinel.init.InitFunc;
import com.alibaba.csp.sentinel.init.InitOrder;
import com.alibaba.csp.sentinel.log.RecordLog;
import com.alibaba.csp.sentinel.slotchain.AbstractLinkedProcessorSlot;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.SlotChainBuilder;
import com.alibaba.csp.sentinel.slotchain.SlotChainProvider;

/**
 * Makes the drop-in deterministic.  SlotChainProvider takes the first non-default SlotChainBuilder ServiceLoader
 * returns (core/slotchain/SlotChainProvider.java:57-75), and the parameter-flow extension registers its own
 * HotParamSlotChainBuilder, so which chain runs would depend on the class-path order.  This InitFunc runs first
 * (InitExecutor runs every InitFunc from Env's static initialiser, before CtSph builds any chain:
 * core/Env.java:33-38, core/init/InitExecutor.java:40-63) and installs {@link GpuSlotChainBuilder} as the
 * provider's resolved builder, then checks that a freshly built chain decides through {@link GpuDecisionSlot}.
 *
 * <p>It never throws.  InitExecutor.doInit catches an InitFunc's exception and stops running every later one
 * (core/init/InitExecutor.java:51-62) -- the parameter extension's callback registration, the transport, the
 * heartbeat -- which would leave a half-initialised process that looks alive.  A failure is instead recorded
 * here ({@link #failure()}), said in the record log and on stderr, and every chain that does reach
 * {@link GpuDecisionSlot} refuses its entries with {@link GpuUnavailableException} (a BlockException, so CtSph
 * exits the entry and rethrows it to the caller: core/CtSph.java:157-166) instead of deciding anything.
 */
@InitOrder(Integer.MIN_VALUE)
public class GpuChainInit implements InitFunc {

    private static volatile String failure;

    /** Why the drop-in is not deciding on the GPU, or null when it is. */
    public static String failure() {
        return failure;
    }

    @Override
    public void init() {
        try {
            install();
        } catch (Throwable t) {   // never through InitExecutor: the other InitFuncs must still run
            fail("GpuChainInit failed", t);
        }
    }

    private static void install() {
        try {
            Field f = SlotChainProvider.class.getDeclaredField("builder");
            f.setAccessible(true);
            Object before = f.get(null);
            if (before != null && !(before instanceof GpuSlotChainBuilder)) {
                RecordLog.warn("[GpuChainInit] replacing the resolved slot chain builder "
                    + before.getClass().getCanonicalName());
            }
            f.set(null, (SlotChainBuilder)new GpuSlotChainBuilder());
        } catch (ReflectiveOperationException | RuntimeException ex) {
            fail("cannot install GpuSlotChainBuilder into SlotChainProvider", ex);
            return;
        }
        ProcessorSlotChain chain = SlotChainProvider.newSlotChain();
        for (AbstractLinkedProcessorSlot<?> s = chain.getNext(); s != null; s = s.getNext()) {
            if (s instanceof GpuDecisionSlot) {
                RecordLog.info("[GpuChainInit] slot chains decide on the GPU (GpuSlotChainBuilder)");
                return;
            }
        }
        fail("the slot chain SlotChainProvider builds has no GpuDecisionSlot", null);
    }

    /** Records the failure (the first one wins) and says so; entries that reach GpuDecisionSlot are refused. */
    static void fail(String msg, Throwable cause) {
        String m = "[sentinel-gpu] " + msg + ": the GPU engine does not decide; GpuDecisionSlot refuses entries";
        if (failure == null) {
            failure = m + (cause == null ? "" : " (" + cause + ")");
        }
        RecordLog.warn(m, cause);
        System.err.println(m);
        if (cause != null) {
            cause.printStackTrace();
        }
    }
}
