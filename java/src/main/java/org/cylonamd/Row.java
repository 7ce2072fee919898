// Row view handed to Table.select predicates (reference java .../Row.java, native Row.cpp:12-81).
package org.cylonamd;

public final class Row {
  private long handle;  // valid only during the predicate call

  Row(long handle) { this.handle = handle; }

  public long getRowIndex() { return nativeIndex(handle); }

  public boolean isNull(int col) { return nativeIsNull(handle, col); }

  public long getInt64(int col) { return nativeGetInt64(handle, col); }

  public double getDouble(int col) { return nativeGetDouble(handle, col); }

  public String getString(int col) { return nativeGetString(handle, col); }

  private static native long nativeIndex(long h);
  private static native boolean nativeIsNull(long h, int col);
  private static native long nativeGetInt64(long h, int col);
  private static native double nativeGetDouble(long h, int col);
  private static native String nativeGetString(long h, int col);
}
