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
 * Same surface as sample/DenseVectorCompressor.java:18-117 with either quantizer on the GPU
 * (Quantizer.newQuantizer's switch, base/Quantizer.java:126-136: QUANTILE or UNIFORM).
 * The compressed state is the packed payload (header, splits, b-bit codes) in a byte[]; its
 * writeObject ships those bytes (b bits per value instead of the reference's 8).
 */
public class HipDenseVectorCompressor implements VectorCompressor {
    private final Quantizer.QuantizationType type;
    private final int binNum;
    private final long seed;
    private int size;
    private byte[] payload;

    public HipDenseVectorCompressor(Quantizer.QuantizationType type, int binNum) {
        this(type, binNum, 0L);
    }

    public HipDenseVectorCompressor(Quantizer.QuantizationType type, int binNum, long seed) {
        if (type != Quantizer.QuantizationType.QUANTILE && type != Quantizer.QuantizationType.UNIFORM)
            throw new SketchMLException("Unrecognizable quantization type: " + type);
        this.type = type;
        this.binNum = binNum;
        this.seed = seed;
    }

    @Override
    public void compressDense(double[] values) {  // DenseVectorCompressor.java:34-41
        size = values.length;
        payload = type == Quantizer.QuantizationType.UNIFORM
                ? HipCodec.encodeDenseUniformF64(HipCodec.ctx(), values, binNum)
                : HipCodec.encodeDenseF64(HipCodec.ctx(), values, binNum, true, seed, 1);
    }

    // DenseVectorCompressor.java:44-55 / 69-81: the dense array is sized maxKey (not maxKey + 1),
    // so the reference throws ArrayIndexOutOfBoundsException at the largest key, and Maths.max of
    // an empty key array throws it too.  Both are kept (INTEGRATION.md §3).
    private static double[] toDense(int[] keys, double[] values) {
        if (keys.length != values.length)
            throw new SketchMLException(String.format(
                    "Lengths of key array and value array do not match: %d, %d", keys.length, values.length));
        if (keys.length == 0)
            throw new ArrayIndexOutOfBoundsException(0);  // Maths.max reads keys[0]
        int maxKey = keys[0];
        for (int k : keys)
            maxKey = Math.max(maxKey, k);
        double[] dense = new double[maxKey];
        for (int i = 0; i < keys.length; i++)
            dense[keys[i]] = values[i];
        return dense;
    }

    @Override
    public void compressSparse(int[] keys, double[] values) {
        compressDense(toDense(keys, values));
    }

    @Override
    public void parallelCompressDense(double[] values) {  // DenseVectorCompressor.java:58-66
        size = values.length;
        // UniformQuantizer.parallelQuantize is quantize's computation (UniformQuantizer.java:48-70)
        payload = type == Quantizer.QuantizationType.UNIFORM
                ? HipCodec.encodeDenseUniformF64(HipCodec.ctx(), values, binNum)
                : HipCodec.encodeDenseF64(HipCodec.ctx(), values, binNum, false, seed,
                        Constants.Parallel.getParallelism());
    }

    @Override
    public void parallelCompressSparse(int[] keys, double[] values) {  // DenseVectorCompressor.java:69-81
        parallelCompressDense(toDense(keys, values));
    }

    @Override
    public double[] decompressDense() {
        double[] out = new double[size];
        HipCodec.decodeDenseF64(HipCodec.ctx(), payload, out);
        return out;
    }

    @Override
    public Pair<int[], double[]> decompressSparse() {
        int[] keys = new int[size];
        Arrays.setAll(keys, i -> i);
        return new ImmutablePair<>(keys, decompressDense());
    }

    @Override
    public void timesBy(double x) {
        HipCodec.timesBy(payload, x);
    }

    @Override
    public double size() {
        return size;
    }

    @Override
    public int memoryBytes() throws IOException {
        return 12 + payload.length;
    }

    private void writeObject(ObjectOutputStream oos) throws IOException {
        oos.writeInt(size);
        oos.writeInt(payload.length);
        oos.write(payload);
    }

    private void readObject(ObjectInputStream ois) throws IOException {
        size = ois.readInt();
        payload = new byte[ois.readInt()];
        ois.readFully(payload);
    }
}
