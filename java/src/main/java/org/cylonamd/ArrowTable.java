// Build a Table from Arrow buffers (J1 ArrowTable; reference arrow/ArrowTable.java:50-141).
// Callers pass the native addresses of Arrow FieldVector buffers (getDataBufferAddress(),
// getValidityBufferAddress(), getOffsetBufferAddress()); the data is copied once into the engine.
package org.cylonamd;

import java.util.ArrayList;
import java.util.List;
import java.util.UUID;

public final class ArrowTable {
  static {
    NativeLoader.load();
  }

  /** cylon Type numbering (cylon_amd.types / C++ Type enum). */
  public static final int INT32 = 6, INT64 = 8, FLOAT = 10, DOUBLE = 11, STRING = 12;

  private final List<String> names = new ArrayList<>();
  private final List<Integer> types = new ArrayList<>();
  private final List<long[]> buffers = new ArrayList<>();  // {data, validity, offsets}
  private final long rows;

  public ArrowTable(long rows) { this.rows = rows; }

  public ArrowTable addColumn(String name, int type, long dataAddress, long validityAddress, long offsetsAddress) {
    names.add(name);
    types.add(type);
    buffers.add(new long[] {dataAddress, validityAddress, offsetsAddress});
    return this;
  }

  public Table finish(CylonContext ctx) {
    int n = names.size();
    int[] t = new int[n];
    long[] d = new long[n], v = new long[n], o = new long[n];
    for (int i = 0; i < n; i++) {
      t[i] = types.get(i);
      d[i] = buffers.get(i)[0];
      v[i] = buffers.get(i)[1];
      o[i] = buffers.get(i)[2];
    }
    String id = UUID.randomUUID().toString();
    CylonContext.check(nativeFromBuffers(id, names.toArray(new String[0]), t, rows, d, v, o));
    return new Table(id, ctx);
  }

  private static native int nativeFromBuffers(String id, String[] names, int[] types, long rows, long[] data,
                                              long[] validity, long[] offsets);
}
