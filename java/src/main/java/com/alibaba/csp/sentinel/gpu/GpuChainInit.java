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
 * If either step fails it says so in the Sentinel record log and on stderr and throws, so a process that would
 * silently run the reference slots on the JVM is visible at start-up.
 */
@InitOrder(Integer.MIN_VALUE)
public class GpuChainInit implements InitFunc {

    @Override
    public void init() throws Exception {
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

    static void fail(String msg, Throwable cause) {
        String m = "[sentinel-gpu] " + msg + ": decisions would run on the JVM slots instead of the GPU engine";
        RecordLog.warn(m, cause);
        System.err.println(m);
        throw new IllegalStateException(m, cause);
    }
}
