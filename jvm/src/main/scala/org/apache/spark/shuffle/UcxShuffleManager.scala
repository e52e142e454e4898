/*
 * org.apache.spark.shuffle.UcxShuffleManager -- the class name the reference's users put in
 * spark.shuffle.manager (README.md:33; the reference's class is
 * shuffle/compat/spark_3_0/UcxShuffleManager.scala:25, constructor (SparkConf, Boolean)), so an
 * existing configuration switches to the MI355X engine without edits.  Everything is
 * GpuUcxShuffleManager's: GPU shuffles for (Long, Long) records under a Hash / Range
 * partitioner, SortShuffleManager's writer and reader for the rest.
 */
package org.apache.spark.shuffle

import org.apache.spark.SparkConf
import org.apache.spark.shuffle.ucx.gpu.GpuUcxShuffleManager

class UcxShuffleManager(conf: SparkConf, isDriver: Boolean) extends GpuUcxShuffleManager(conf, isDriver)
