package org.cylonamd;

/** Loads libcylon_jni (which links the cylon_amd native library). */
final class NativeLoader {
  private static boolean loaded = false;

  static synchronized void load() {
    if (!loaded) {
      System.loadLibrary("cylon_jni");
      loaded = true;
    }
  }

  private NativeLoader() {}
}
