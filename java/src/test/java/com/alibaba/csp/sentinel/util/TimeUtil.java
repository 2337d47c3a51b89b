package com.alibaba.csp.sentinel.util;

/**
 * Test-scope stand-in for the reference's TimeUtil (core/util/TimeUtil.java:25-52), first on the test
 * class path: the replay harness sets the clock to each event's ts instead of a 1 ms tick thread, so
 * the unmodified slots see exactly the trace's time.
 */
public final class TimeUtil {

    private static volatile long now;

    private TimeUtil() {}

    public static long currentTimeMillis() {
        return now;
    }

    public static void set(long ms) {
        now = ms;
    }
}
