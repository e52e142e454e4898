/*
 * Thrown by SgxNative (jni/sgx_jni.c) for SGX_ERR_NOT_FOUND, SGX_ERR_COMM and SGX_ERR_TIMEOUT:
 * a block that is not there, a failed collective, a peer that stopped answering.
 * GpuShuffleClient turns it into BlockFetchingListener.onBlockFetchFailure, so Spark raises
 * FetchFailedException and retries the stage -- the reference's client never reports a
 * failed fetch (spark_3_0/UcxShuffleClient.scala:36-40) and spins forever on a dead peer
 * (:44-46).
 */
package org.apache.spark.shuffle.ucx.gpu;

public class SgxFetchException extends RuntimeException {
  public SgxFetchException(String message) {
    super(message);
  }
}
