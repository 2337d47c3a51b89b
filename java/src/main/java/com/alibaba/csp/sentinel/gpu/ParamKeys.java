package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.JAVA_LONG;

/**
 * Interned 64-bit keys of parameter values: {@code sg_param_key(text, classType)}, the typing of
 * ParamFlowRuleUtil.parseItemValue (param/slots/block/flow/param/ParamFlowRuleUtil.java:85-121), so
 * that a hot item {@code ("1", "int")} and a call argument {@code Integer 1} meet on one key while
 * {@code Long 1} and {@code "1"} stay different (the reference's CLHM compares with equals()).
 *
 * <p>The boxed types a hot item can name are interned by their text; any other class (which the
 * reference compares with its own equals/hashCode) by class name + toString, a documented
 * approximation: two objects of such a class with equal toString() share a key.
 */
final class ParamKeys {

    private ParamKeys() {}

    static long of(Object v) {
        final String text;
        final String type;
        if (v instanceof String) {
            text = (String)v;
            type = "java.lang.String";
        } else if (v instanceof Integer) {
            text = v.toString();
            type = "java.lang.Integer";
        } else if (v instanceof Long) {
            text = v.toString();
            type = "java.lang.Long";
        } else if (v instanceof Double) {
            text = v.toString();     // Double.toString round-trips through strtod exactly
            type = "java.lang.Double";
        } else if (v instanceof Float) {
            text = v.toString();
            type = "java.lang.Float";
        } else if (v instanceof Byte) {
            text = v.toString();
            type = "java.lang.Byte";
        } else if (v instanceof Short) {
            text = v.toString();
            type = "java.lang.Short";
        } else if (v instanceof Boolean) {
            text = v.toString();
            type = "java.lang.Boolean";
        } else if (v instanceof Character) {
            text = v.toString();
            type = "char";
        } else {
            text = v.getClass().getName() + "\u0001" + v;
            type = "java.lang.String";
        }
        try (Arena a = Arena.ofConfined()) {
            MemorySegment out = a.allocate(JAVA_LONG);
            int rc = (int)SentinelGpu.PARAM_KEY.invokeExact(MemorySegment.NULL, a.allocateFrom(text),
                                                            a.allocateFrom(type), out);
            SentinelGpu.check(rc);
            return out.get(JAVA_LONG, 0);
        } catch (RuntimeException e) {
            throw e;
        } catch (Throwable t) {
            throw new IllegalStateException(t);
        }
    }
}
