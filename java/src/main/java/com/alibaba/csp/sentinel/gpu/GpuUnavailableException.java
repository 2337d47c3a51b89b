package com.alibaba.csp.sentinel.gpu;

import com.alibaba.csp.sentinel.slots.block.BlockException;

/**
 * An entry refused because the drop-in could not take over the decision path (GpuChainInit recorded a
 * failure, or the engine could not be created).  A BlockException, so CtSph exits the entry and rethrows it
 * to the caller (core/CtSph.java:157-166): the request fails closed and visibly, instead of passing without
 * any rule being checked.
 */
public class GpuUnavailableException extends BlockException {

    public GpuUnavailableException(String reason) {
        super("sentinel-gpu", reason);
    }

    @Override
    public Throwable fillInStackTrace() {
        return this;
    }
}
