// Reference: java/src/main/java/org/cylondata/cylon/ops/JoinConfig.java
package org.cylonamd;

public final class JoinConfig {
  public enum Type { INNER, LEFT, RIGHT, FULL_OUTER }
  public enum Algorithm { SORT, HASH }

  final int leftIndex;
  final int rightIndex;
  final Type type;
  final Algorithm algorithm;

  public JoinConfig(int leftIndex, int rightIndex) {
    this(leftIndex, rightIndex, Type.INNER, Algorithm.SORT);
  }

  public JoinConfig(int leftIndex, int rightIndex, Type type, Algorithm algorithm) {
    this.leftIndex = leftIndex;
    this.rightIndex = rightIndex;
    this.type = type;
    this.algorithm = algorithm;
  }

  public JoinConfig joinType(Type t) { return new JoinConfig(leftIndex, rightIndex, t, algorithm); }

  public JoinConfig useAlgorithm(Algorithm a) { return new JoinConfig(leftIndex, rightIndex, type, a); }
}
