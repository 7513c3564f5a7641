package org.dma.sketchml.hip;

import org.apache.commons.lang3.tuple.ImmutablePair;
import org.apache.commons.lang3.tuple.Pair;
import org.dma.sketchml.sketch.base.Quantizer;
import org.dma.sketchml.sketch.base.SketchMLException;
import org.dma.sketchml.sketch.base.VectorCompressor;
import org.dma.sketchml.sketch.common.Constants;

import java.io.IOException;
import java.io.ObjectInputStream;
import java.io.ObjectOutputStream;
import java.util.Arrays;

/**
 * Same surface as sample/SparseVectorCompressor.java:18-148: quantize the values, then
 * GroupedMinMaxSketch.create over (keys, bins) -- group partition, MinMaxSketch tables,
 * DeltaAdaptiveEncoder keys -- on the GPU.  The double values are quantised as doubles (the
 * sketch samples and bins are those of the reference's double[] path) and decompressSparse returns
 * quantValues[bin] in double.  writeObject ships the GroupedMinMaxSketch field stream (HuffmanEncoder
 * tables, BitSet words) and quantValues.
 */
public class HipSparseVectorCompressor implements VectorCompressor, AutoCloseable {
    private final Quantizer.QuantizationType quantType;
    private final int quantBinNum, groupNum, rowNum;
    private final double colRatio;
    private final long seed, hashSeed;
    private int size;
    private transient long handle;
    private double[] quantValues;

    public HipSparseVectorCompressor(Quantizer.QuantizationType quantType, int quantBinNum, int groupNum,
                                     int rowNum, double colRatio) {
        this(quantType, quantBinNum, groupNum, rowNum, colRatio, 0L, 0L);
    }

    public HipSparseVectorCompressor(Quantizer.QuantizationType quantType, int quantBinNum, int groupNum,
                                     int rowNum, double colRatio, long seed, long hashSeed) {
        this.quantType = quantType;
        this.quantBinNum = quantBinNum;
        this.groupNum = groupNum;
        this.rowNum = rowNum;
        this.colRatio = colRatio;
        this.seed = seed;
        this.hashSeed = hashSeed;
    }

    private void encode(int[] keys, double[] values, int parallelism) {
        if (keys.length != values.length)
            throw new SketchMLException(String.format(
                    "Lengths of key array and value array do not match: %d, %d", keys.length, values.length));
        close();
        size = keys.length;
        handle = HipCodec.encodeSparse(HipCodec.ctx(), keys, values, quantBinNum, groupNum, rowNum,
                colRatio, seed, hashSeed, quantType == Quantizer.QuantizationType.UNIFORM, parallelism);
        quantValues = HipCodec.sparseValues(handle, quantBinNum);
    }

    @Override
    public void compressDense(double[] values) {
        int[] keys = new int[values.length];
        Arrays.setAll(keys, i -> i);
        compressSparse(keys, values);
    }

    @Override
    public void compressSparse(int[] keys, double[] values) {
        encode(keys, values, 1);
    }

    @Override
    public void parallelCompressDense(double[] values) {
        int[] keys = new int[values.length];
        Arrays.setAll(keys, i -> i);
        parallelCompressSparse(keys, values);
    }

    @Override
    public void parallelCompressSparse(int[] keys, double[] values) {
        encode(keys, values, Constants.Parallel.getParallelism());
    }

    @Override
    public double[] decompressDense() {  // SparseVectorCompressor.java:106-114: maxKey + 1 entries
        Pair<int[], double[]> kv = decompressSparse();
        int maxKey = 0;
        for (int k : kv.getLeft())
            maxKey = Math.max(k, maxKey);
        double[] res = new double[maxKey + 1];
        for (int i = 0; i < kv.getLeft().length; i++)
            res[kv.getLeft()[i]] = kv.getRight()[i];
        return res;
    }

    @Override
    public Pair<int[], double[]> decompressSparse() {
        // sized by the payload itself (a deserialised `size` field may disagree with the stream)
        final int nnz = HipCodec.sparseNnz(handle);
        int[] keys = new int[nnz];
        double[] values = new double[nnz];
        HipCodec.decodeSparse(HipCodec.ctx(), handle, keys, values);
        return new ImmutablePair<>(keys, values);
    }

    @Override
    public void timesBy(double x) {
        HipCodec.sparseTimesBy(handle, x);
        quantValues = HipCodec.sparseValues(handle, quantBinNum);
    }

    @Override
    public double size() {
        return size;
    }

    @Override
    public int memoryBytes() throws IOException {  // SparseVectorCompressor.java:142-147
        return 28 + quantValues.length * 8 + HipCodec.writeSparse(HipCodec.ctx(), handle).length;
    }

    @Override
    public void close() {
        if (handle != 0) {
            HipCodec.freeSparse(handle);
            handle = 0;
        }
    }

    private void writeObject(ObjectOutputStream oos) throws IOException {
        oos.defaultWriteObject();
        byte[] stream = HipCodec.writeSparse(HipCodec.ctx(), handle);
        oos.writeInt(stream.length);
        oos.write(stream);
    }

    private void readObject(ObjectInputStream ois) throws IOException, ClassNotFoundException {
        ois.defaultReadObject();
        byte[] stream = new byte[ois.readInt()];
        ois.readFully(stream);
        handle = HipCodec.readSparse(HipCodec.ctx(), stream, quantValues);
    }
}
