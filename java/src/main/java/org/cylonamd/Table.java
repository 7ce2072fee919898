// Java Table (J1).  Reference: java/src/main/java/org/cylondata/cylon/Table.java:47-293.
// A Table is a string ID into the native registry (C28); every operation creates a new ID.
package org.cylonamd;

import java.util.UUID;
import java.util.function.Predicate;

public class Table {
  static {
    NativeLoader.load();
  }

  private final String id;
  private final CylonContext ctx;

  Table(String id, CylonContext ctx) {
    this.id = id;
    this.ctx = ctx;
  }

  private static String newId() { return UUID.randomUUID().toString(); }

  public String getId() { return id; }

  public static Table fromCSV(CylonContext ctx, String path) {
    String id = newId();
    CylonContext.check(nativeReadCSV(path, id));
    return new Table(id, ctx);
  }

  public void writeCSV(String path) { CylonContext.check(nativeWriteCSV(id, path)); }

  public long getRowCount() { return nativeRowCount(id); }

  public int getColumnCount() { return nativeColumnCount(id); }

  public Table join(Table right, JoinConfig cfg) { return joinImpl(right, cfg, false); }

  public Table distributedJoin(Table right, JoinConfig cfg) { return joinImpl(right, cfg, true); }

  private Table joinImpl(Table right, JoinConfig cfg, boolean distributed) {
    String out = newId();
    CylonContext.check(nativeJoin(id, right.id, cfg.type.ordinal(), cfg.algorithm.ordinal(), cfg.leftIndex,
        cfg.rightIndex, distributed, out));
    return new Table(out, ctx);
  }

  public Table union(Table other) { return setOp(other, 0, false); }

  public Table subtract(Table other) { return setOp(other, 1, false); }

  public Table intersect(Table other) { return setOp(other, 2, false); }

  public Table distributedUnion(Table other) { return setOp(other, 0, true); }

  private Table setOp(Table other, int op, boolean distributed) {
    String out = newId();
    CylonContext.check(nativeSetOp(id, other.id, op, distributed, out));
    return new Table(out, ctx);
  }

  public Table sort(int column) { return sort(column, true); }

  public Table sort(int column, boolean ascending) {
    String out = newId();
    CylonContext.check(nativeSort(id, column, ascending, out));
    return new Table(out, ctx);
  }

  public Table project(int[] columns) {
    String out = newId();
    CylonContext.check(nativeProject(id, columns, out));
    return new Table(out, ctx);
  }

  public static Table merge(CylonContext ctx, Table... tables) {
    String[] ids = new String[tables.length];
    for (int i = 0; i < tables.length; i++) ids[i] = tables[i].id;
    String out = newId();
    CylonContext.check(nativeMerge(ids, out));
    return new Table(out, ctx);
  }

  /** Rows for which the predicate holds (reference Table.select over Row). */
  public Table select(Predicate<Row> predicate) {
    String out = newId();
    CylonContext.check(nativeSelect(id, predicate, out));
    return new Table(out, ctx);
  }

  public void print() { print(0, -1); }

  public void print(long from, long to) { CylonContext.check(nativePrint(id, from, to)); }

  /** Reference: hash/round-robin partition through the Java API are unsupported (Table.java:167-182). */
  public Table[] hashPartition(int[] columns, int partitions) {
    throw new UnsupportedOperationException("hashPartition is not supported through the Java API");
  }

  public Table[] roundRobinPartition(int partitions) {
    throw new UnsupportedOperationException("roundRobinPartition is not supported through the Java API");
  }

  public void clear() { CylonContext.check(nativeRemove(id)); }

  private static native int nativeReadCSV(String path, String id);
  private static native int nativeWriteCSV(String id, String path);
  private static native long nativeRowCount(String id);
  private static native int nativeColumnCount(String id);
  private static native int nativeJoin(String l, String r, int type, int algorithm, int lc, int rc, boolean dist,
                                       String out);
  private static native int nativeSetOp(String a, String b, int op, boolean dist, String out);
  private static native int nativeSort(String id, int col, boolean asc, String out);
  private static native int nativeProject(String id, int[] cols, String out);
  private static native int nativeMerge(String[] ids, String out);
  private static native int nativeSelect(String id, Predicate<Row> pred, String out);
  private static native int nativePrint(String id, long from, long to);
  private static native int nativeRemove(String id);
}
