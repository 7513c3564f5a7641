package org.dma.sketchml.hip;

/**
 * Natives of jni/skml_jni.c, one per C entry point of include/skml.h they wrap.  A context is one
 * HIP stream on one GPU (skml_ctx); dense payloads travel as byte[] (header, splits, packed codes),
 * sparse payloads stay on the device behind a handle.
 */
final class HipCodec {
    static {
        System.loadLibrary("skml_jni");
    }

    private HipCodec() {
    }

    static native long ctxCreate(int device);

    static native void ctxDestroy(long ctx);

    // QuantileQuantizer.quantize / parallelQuantize (parallelism > 1) over float[] / double[]
    static native byte[] encodeDense(long ctx, float[] x, int binNum, boolean dedup, long seed, int parallelism);

    static native byte[] encodeDenseF64(long ctx, double[] x, int binNum, boolean dedup, long seed,
                                        int parallelism);

    // UniformQuantizer.quantize / parallelQuantize (the same computation) over double[]
    static native byte[] encodeDenseUniformF64(long ctx, double[] x, int binNum);

    static native void decodeDense(long ctx, byte[] payload, float[] out);

    static native void decodeDenseF64(long ctx, byte[] payload, double[] out);

    static native void getBins(byte[] payload, int[] out);

    /** {binNum, n, zeroIdx, min, max, splits...} */
    static native double[] info(byte[] payload);

    static native void timesBy(byte[] payload, double x);

    // SparseVectorCompressor: quantize(values) + GroupedMinMaxSketch.create(keys, bins)
    static native long encodeSparse(long ctx, int[] keys, double[] vals, int binNum, int groupNum, int rowNum,
                                    double colRatio, long seed, long hashSeed, boolean uniform, int parallelism);

    /** keys and quantValues[bin] as doubles; both arrays must hold sparseNnz(sparse) entries */
    static native void decodeSparse(long ctx, long sparse, int[] keys, double[] vals);

    static native int sparseNnz(long sparse);

    static native double[] sparseValues(long sparse, int binNum);

    static native void sparseTimesBy(long sparse, double x);

    static native byte[] writeSparse(long ctx, long sparse);

    static native long readSparse(long ctx, byte[] stream, double[] quantValues);

    static native void freeSparse(long sparse);

    // DeltaAdaptiveEncoder as a BinaryEncoder
    /** {numIntervals, flagKind, nFlagBits, nDeltaBits, nFlagWords, nDeltaWords, flagWords..., deltaWords...} */
    static native long[] deltaEncode(long ctx, int[] keys);

    static native int[] deltaDecode(long ctx, int size, int numIntervals, boolean flagKind, long[] flagWords,
                                    long[] deltaWords);

    /** One context per thread (a context is not re-entrant, include/skml.h), on GPU 0 unless set. */
    private static final ThreadLocal<Long> CTX = ThreadLocal.withInitial(
            () -> ctxCreate(Integer.getInteger("sketchml.hip.device", 0)));

    static long ctx() {
        return CTX.get();
    }
}
