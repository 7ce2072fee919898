// Java API of cylon_amd (J1).  Reference surface: java/src/main/java/org/cylondata/cylon/
// CylonContext.java:24-84.  Native methods are implemented in
// java/src/main/native/cylon_jni.cpp over the C ABI (cylon_amd/include/cylon_capi.h).
package org.cylonamd;

public final class CylonContext {
  static {
    NativeLoader.load();
  }

  private CylonContext() {}

  /** Local context on "cpu" or "cuda:<i>". */
  public static CylonContext init(String device) {
    check(nativeInit(device));
    return new CylonContext();
  }

  public static CylonContext init() {
    return init("cpu");
  }

  /**
   * Distributed context from the torchrun environment (RANK, WORLD_SIZE, MASTER_ADDR,
   * MASTER_PORT, LOCAL_RANK): "rccl" (one GPU per rank), "tcp" (host tables) or "mpi".
   * Reference: CylonContext.init(MPIConfig) / InitDistributed.
   */
  public static CylonContext initDistributed(String commType) {
    check(nativeInitDistributed(commType));
    return new CylonContext();
  }

  public int getRank() { return nativeRank(); }

  public int getWorldSize() { return nativeWorldSize(); }

  public void barrier() { check(nativeBarrier()); }

  public void finalizeCtx() { check(nativeFinalize()); }

  static void check(int code) {
    if (code != 0) throw new CylonException(code, nativeLastError());
  }

  private static native int nativeInit(String device);
  private static native int nativeInitDistributed(String commType);
  private static native int nativeRank();
  private static native int nativeWorldSize();
  private static native int nativeBarrier();
  private static native int nativeFinalize();
  static native String nativeLastError();
}
