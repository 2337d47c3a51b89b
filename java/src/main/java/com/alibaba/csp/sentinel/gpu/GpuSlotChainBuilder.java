package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slotchain.DefaultProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.ProcessorSlotChain;
import com.alibaba.csp.sentinel.slotchain.SlotChainBuilder;
import com.alibaba.csp.sentinel.slots.clusterbuilder.ClusterBuilderSlot;
import com.alibaba.csp.sentinel.slots.logger.LogSlot;
import com.alibaba.csp.sentinel.slots.nodeselector.NodeSelectorSlot;

/**
 * The drop-in: picked up by SlotChainProvider through
 * META-INF/services/com.alibaba.csp.sentinel.slotchain.SlotChainBuilder (core/slotchain/SlotChainProvider.java)
 * in place of HotParamSlotChainBuilder (param/slots/HotParamSlotChainBuilder.java:38-51).  The node-building
 * and logging slots are the reference's own; the six deciding slots are {@link GpuDecisionSlot}.
 */
public class GpuSlotChainBuilder implements SlotChainBuilder {

    @Override
    public ProcessorSlotChain build() {
        ProcessorSlotChain chain = new DefaultProcessorSlotChain();
        chain.addLast(new NodeSelectorSlot());
        chain.addLast(new ClusterBuilderSlot());
        chain.addLast(new LogSlot());
        chain.addLast(new GpuDecisionSlot());
        return chain;
    }
}
