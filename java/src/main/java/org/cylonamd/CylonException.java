package org.cylonamd;

/** A failed cylon operation: the cylon Code and message (reference Status). */
public final class CylonException extends RuntimeException {
  private final int code;

  public CylonException(int code, String message) {
    super("cylon error " + code + ": " + message);
    this.code = code;
  }

  public int getCode() { return code; }
}
