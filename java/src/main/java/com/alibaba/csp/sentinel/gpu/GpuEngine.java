package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.reflect.Array;
import java.util.ArrayList;
import java.util.Collection;
import java.util.List;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.LinkedBlockingQueue;
import java.util.concurrent.TimeUnit;
import java.util.concurrent.locks.LockSupport;

import com.alibaba.csp.sentinel.config.SentinelConfig;
import com.alibaba.csp.sentinel.node.IntervalProperty;
import com.alibaba.csp.sentinel.node.SampleCountProperty;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

/**
 * The process-wide engine and its batcher.  Calling threads enqueue one {@link Op} per SphU.entry /
 * Entry.exit / Tracer.trace; a single batcher thread drains the queue in arrival order, gives each op
 * its global event index (the {@code ref} an EXIT names), clamps timestamps to non-decreasing order,
 * writes the sg_event / sg_event_ext / sg_arg arrays and calls {@code sg_submit_ex}.  ENTRY callers
 * park until their decision word is back; EXIT / TRACE callers do not wait.
 *
 * <p>This replaces the per-call slot walk of CtSph.entryWithPriority (core/CtSph.java:116-150): the
 * decisions are those of the reference for the same event order, taken for the whole batch on the GPU.
 * Every native call is made under {@link #nativeLock}; the engine handle is not shared across threads
 * otherwise.  A failing sg_submit_ex fails every ENTRY of its batch with the library's message -- there
 * is no Java fallback that would decide instead.
 */
final class GpuEngine {

    /** One event.  {@code decision} is written by the batcher before it unparks {@code waiter}. */
    static final class Op {
        final long ts;
        final int resId;
        final int count;
        final int kind;
        final int flags;
        final long aux;
        final int origin;
        final int context;
        final Object[] args;
        final Thread waiter;
        long gidx = -1;
        volatile int decision = -1;
        volatile String error;

        Op(long ts, int resId, int count, int kind, int flags, long aux, int origin, int context, Object[] args,
           Thread waiter) {
            this.ts = ts;
            this.resId = resId;
            this.count = count;
            this.kind = kind;
            this.flags = flags;
            this.aux = aux;
            this.origin = origin;
            this.context = context;
            this.args = args;
            this.waiter = waiter;
        }
    }

    private static volatile GpuEngine instance;

    static GpuEngine get() {
        GpuEngine e = instance;
        if (e == null) {
            synchronized (GpuEngine.class) {
                e = instance;
                if (e == null) {
                    e = new GpuEngine();
                    instance = e;
                }
            }
        }
        return e;
    }

    final Object nativeLock = new Object();
    final MemorySegment handle;
    private final int maxBatch;
    private final LinkedBlockingQueue<Op> queue = new LinkedBlockingQueue<>();
    private final ConcurrentHashMap<String, Integer> resIds = new ConcurrentHashMap<>();
    private final ConcurrentHashMap<String, Integer> originIds = new ConcurrentHashMap<>();
    private final ConcurrentHashMap<String, Integer> contextIds = new ConcurrentHashMap<>();
    private final Thread batcher;

    // batcher-thread state
    private long nextGidx;
    private long lastTs = Long.MIN_VALUE;
    private boolean poisoned;
    private final Arena arena = Arena.ofShared();
    private MemorySegment evBuf, extBuf, outBuf, argBuf;
    private int evCap, argCap;

    private GpuEngine() {
        final java.lang.foreign.StructLayout C = SentinelGpu.SG_CONFIG;
        MemorySegment cfg = arena.allocate(C);
        try {
            SentinelGpu.CONFIG_DEFAULT.invokeExact(cfg);
            // the reference's own process-wide settings
            cfg.set(JAVA_INT, off(C, "sample_count"), SampleCountProperty.SAMPLE_COUNT);
            cfg.set(JAVA_INT, off(C, "interval_ms"), IntervalProperty.INTERVAL);
            cfg.set(JAVA_INT, off(C, "cold_factor"), SentinelConfig.coldFactor());
            cfg.set(JAVA_INT, off(C, "statistic_max_rt"), SentinelConfig.statisticMaxRt());
            cfg.set(JAVA_INT, off(C, "device"), Integer.getInteger("sentinel.gpu.device", 0));
            Integer maxRes = Integer.getInteger("sentinel.gpu.maxResources");
            if (maxRes != null) {
                cfg.set(JAVA_INT, off(C, "max_resources"), maxRes);
            }
            maxBatch = Math.min(Integer.getInteger("sentinel.gpu.maxBatch", 1 << 16),
                                cfg.get(JAVA_INT, off(C, "max_batch_events")));
            MemorySegment out = arena.allocate(ADDRESS);
            SentinelGpu.check((int)SentinelGpu.ENGINE_CREATE.invokeExact(cfg, out));
            handle = out.get(ADDRESS, 0);
        } catch (RuntimeException ex) {
            throw ex;
        } catch (Throwable t) {
            throw new IllegalStateException("sentinel_gpu: engine creation failed", t);
        }
        batcher = new Thread(this::loop, "sentinel-gpu-batcher");
        batcher.setDaemon(true);
        batcher.start();
        GpuRuleSync.attach(this);
    }

    private static long off(java.lang.foreign.StructLayout l, String f) {
        return l.byteOffset(MemoryLayout.PathElement.groupElement(f));
    }

    // ---- interning (any thread)
    int resourceId(String name) {
        return resIds.computeIfAbsent(name, n -> {
            synchronized (nativeLock) {
                try (Arena a = Arena.ofConfined()) {
                    MemorySegment names = a.allocate(ADDRESS);
                    names.set(ADDRESS, 0, a.allocateFrom(n));
                    MemorySegment id = a.allocate(JAVA_INT);
                    SentinelGpu.check((int)SentinelGpu.REGISTER_RESOURCES.invokeExact(handle, names, 1, id));
                    return id.get(JAVA_INT, 0);
                } catch (RuntimeException ex) {
                    throw ex;
                } catch (Throwable t) {
                    throw new IllegalStateException(t);
                }
            }
        });
    }

    int originId(String origin) {
        if (origin == null || origin.isEmpty()) {
            return 0;
        }
        return originIds.computeIfAbsent(origin, o -> intern(SentinelGpu.INTERN_ORIGIN, o));
    }

    int contextId(String name) {
        return contextIds.computeIfAbsent(name, c -> intern(SentinelGpu.INTERN_CONTEXT, c));
    }

    private int intern(java.lang.invoke.MethodHandle fn, String s) {
        synchronized (nativeLock) {
            try (Arena a = Arena.ofConfined()) {
                MemorySegment id = a.allocate(JAVA_INT);
                SentinelGpu.check((int)fn.invokeExact(handle, a.allocateFrom(s), id));
                return id.get(JAVA_INT, 0);
            } catch (RuntimeException ex) {
                throw ex;
            } catch (Throwable t) {
                throw new IllegalStateException(t);
            }
        }
    }

    // ---- events
    /** Enqueue an ENTRY and park until the batcher has its decision word. */
    int decide(Op op) {
        queue.add(op);
        while (op.decision == -1 && op.error == null) {
            LockSupport.park(this);
        }
        if (op.error != null) {
            throw new IllegalStateException(op.error);
        }
        return op.decision;
    }

    /** Global event index of a decided ENTRY (valid once {@link #decide} returned). */
    static long indexOf(Op entry) {
        return entry.gidx;
    }

    /** EXIT / TRACE: ordered behind every op enqueued before it, no wait. */
    void post(Op op) {
        queue.add(op);
    }

    private void loop() {
        List<Op> batch = new ArrayList<>();
        while (true) {
            try {
                Op first = queue.poll(50, TimeUnit.MILLISECONDS);
                if (first == null) {
                    continue;
                }
                batch.add(first);
                queue.drainTo(batch, maxBatch - 1);
                GpuRuleSync.rehook();
                submit(batch);
            } catch (InterruptedException ie) {
                return;
            } catch (Throwable t) {
                String msg = "sentinel_gpu: batch failed: " + t.getMessage();
                for (Op op : batch) {
                    op.error = msg;
                    if (op.waiter != null) {
                        LockSupport.unpark(op.waiter);
                    }
                }
            } finally {
                batch.clear();
            }
        }
    }

    /**
     * The op's arguments with every Collection / array copied once: the slot count and the table fill read the same
     * elements even if a caller's collection changes meanwhile.
     */
    private static Object[] argSnapshot(Op op) {
        if (op.args == null) {
            return null;
        }
        int n = Math.min(op.args.length, SentinelGpu.MAX_ARGS);
        Object[] a = new Object[n];
        for (int i = 0; i < n; i++) {
            Object v = op.args[i];
            if (v instanceof Collection) {
                a[i] = ((Collection<?>)v).toArray();
            } else if (v != null && v.getClass().isArray()) {
                int len = Array.getLength(v);
                Object[] el = new Object[len];
                for (int j = 0; j < len; j++) {
                    el[j] = Array.get(v, j);
                }
                a[i] = el;
            } else {
                a[i] = v;
            }
        }
        return a;
    }

    private static int argSlots(Object[] a) {
        if (a == null) {
            return 0;
        }
        int slots = a.length;
        for (Object v : a) {
            if (v instanceof Object[]) {
                slots += ((Object[])v).length;
            }
        }
        return slots;
    }

    private void ensure(int nEv, int nArg) {
        if (nEv > evCap) {
            evCap = Math.max(nEv, evCap * 2);
            evBuf = arena.allocate(SentinelGpu.SG_EVENT, evCap);
            extBuf = arena.allocate(SentinelGpu.SG_EVENT_EXT, evCap);
            outBuf = arena.allocate(JAVA_INT, evCap);
        }
        if (nArg > argCap) {
            argCap = Math.max(nArg, Math.max(64, argCap * 2));
            argBuf = arena.allocate(SentinelGpu.SG_ARG, argCap);
        }
    }

    private static final java.lang.foreign.StructLayout EV = SentinelGpu.SG_EVENT;
    private static final java.lang.foreign.StructLayout EXT = SentinelGpu.SG_EVENT_EXT;
    private static final java.lang.foreign.StructLayout ARG = SentinelGpu.SG_ARG;
    private static final long EV_SZ = EV.byteSize(), EXT_SZ = EXT.byteSize(), ARG_SZ = ARG.byteSize();
    private static final long EV_TS = off(EV, "ts"), EV_RES = off(EV, "res_id"), EV_COUNT = off(EV, "count"),
        EV_KIND = off(EV, "kind"), EV_FLAGS = off(EV, "flags"), EV_AUX = off(EV, "aux");
    private static final long X_ORIGIN = off(EXT, "origin_id"), X_CONTEXT = off(EXT, "context_id"),
        X_OFF = off(EXT, "arg_off"), X_N = off(EXT, "n_args");
    private static final long A_KEY = off(ARG, "key"), A_KIND = off(ARG, "kind"), A_LEN = off(ARG, "len");

    private void putArg(int slot, Object v) {
        long o = slot * ARG_SZ;
        if (v == null) {
            argBuf.set(JAVA_LONG, o + A_KEY, 0L);
            argBuf.set(JAVA_INT, o + A_KIND, SentinelGpu.ARG_NULL);
        } else {
            argBuf.set(JAVA_LONG, o + A_KEY, ParamKeys.of(v));
            argBuf.set(JAVA_INT, o + A_KIND, SentinelGpu.ARG_SCALAR);
        }
        argBuf.set(JAVA_INT, o + A_LEN, 0);
    }

    private void submit(List<Op> batch) throws Throwable {
        if (poisoned) {
            throw new IllegalStateException("an earlier batch failed; the engine's event indices are unknown");
        }
        int n = batch.size();
        Object[][] args = new Object[n][];
        int nArg = 0;
        for (int i = 0; i < n; i++) {
            args[i] = argSnapshot(batch.get(i));
            nArg += argSlots(args[i]);
        }
        ensure(n, nArg);
        // Fill the buffers first: a caller's toString() may throw in ParamKeys.of, and then nothing of this batch
        // reached the engine -- no event index is consumed and later batches stay valid.
        int tail = 0;
        long ts0 = lastTs;
        for (int i = 0; i < n; i++) {
            Op op = batch.get(i);
            long ts = Math.max(op.ts, ts0);
            ts0 = ts;
            long e = i * EV_SZ;
            evBuf.set(JAVA_LONG, e + EV_TS, ts);
            evBuf.set(JAVA_INT, e + EV_RES, op.resId);
            evBuf.set(JAVA_SHORT, e + EV_COUNT, (short)op.count);
            evBuf.set(JAVA_BYTE, e + EV_KIND, (byte)op.kind);
            evBuf.set(JAVA_BYTE, e + EV_FLAGS, (byte)op.flags);
            evBuf.set(JAVA_LONG, e + EV_AUX, op.aux);
            Object[] a = args[i];
            int na = a == null ? 0 : a.length;
            long x = i * EXT_SZ;
            extBuf.set(JAVA_INT, x + X_ORIGIN, op.origin);
            extBuf.set(JAVA_INT, x + X_CONTEXT, op.context);
            extBuf.set(JAVA_INT, x + X_OFF, tail);
            extBuf.set(JAVA_INT, x + X_N, na);
            int base = tail;
            tail += na;
            for (int k = 0; k < na; k++) {
                Object v = a[k];
                if (v instanceof Object[]) {
                    int start = tail;
                    for (Object el : (Object[])v) {
                        putArg(tail++, el);
                    }
                    long o = (base + k) * ARG_SZ;
                    argBuf.set(JAVA_LONG, o + A_KEY, start);
                    argBuf.set(JAVA_INT, o + A_KIND, SentinelGpu.ARG_LIST);
                    argBuf.set(JAVA_INT, o + A_LEN, tail - start);
                } else {
                    putArg(base + k, v);
                }
            }
        }
        int rc;
        synchronized (nativeLock) {
            rc = (int)SentinelGpu.SUBMIT_EX.invokeExact(handle, evBuf, extBuf, (long)n,
                                                        tail == 0 ? MemorySegment.NULL : argBuf, (long)tail, outBuf);
        }
        if (rc != SentinelGpu.SG_OK) {
            // whether the engine counted the rejected batch depends on where it failed: the event indices
            // (EXIT refs) are no longer known, so every later batch fails too
            poisoned = true;
            SentinelGpu.check(rc);
        }
        // the batch is in: its events hold the next n global indices (EXIT / TRACE references name them)
        lastTs = ts0;
        for (int i = 0; i < n; i++) {
            batch.get(i).gidx = nextGidx + i;
        }
        nextGidx += n;
        for (int i = 0; i < n; i++) {
            Op op = batch.get(i);
            if (op.waiter != null) {
                op.decision = outBuf.getAtIndex(JAVA_INT, i);
                LockSupport.unpark(op.waiter);
            }
        }
    }

    /** A MetricNode snapshot of every resource at {@code now} (sg_snapshot_metrics). */
    MemorySegment snapshot(long now, Arena into, int cap) {
        synchronized (nativeLock) {
            MemorySegment rows = into.allocate(SentinelGpu.SG_METRIC_NODE, Math.max(1, cap));
            MemorySegment n = into.allocate(JAVA_LONG);
            try {
                SentinelGpu.check((int)SentinelGpu.SNAPSHOT_METRICS.invokeExact(handle, now, rows, (long)cap, n));
            } catch (RuntimeException ex) {
                throw ex;
            } catch (Throwable t) {
                throw new IllegalStateException(t);
            }
            return rows.asSlice(0, Math.min(cap, n.get(JAVA_LONG, 0)) * SentinelGpu.SG_METRIC_NODE.byteSize());
        }
    }
}
