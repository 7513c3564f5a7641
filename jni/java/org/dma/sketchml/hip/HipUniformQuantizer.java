package org.dma.sketchml.hip;

import org.dma.sketchml.sketch.base.Quantizer;

/**
 * Drop-in for quantization/UniformQuantizer.java:21-70: min / max (Double.MAX_VALUE /
 * Double.MIN_VALUE initialised), binNum - 1 splits by repeated {@code += (max - min) / binNum},
 * findZeroIdx and the bins, computed on the GPU (skml_dense_encode_uniform_f64 through the host
 * entry point).  The same Quantizer fields are filled as by HipQuantileQuantizer, so Quantizer's
 * getValues / indexOf / writeObject / readObject work unchanged.  parallelQuantize is quantize's
 * computation, as in the reference (its slices only parallelise quantizeToBins).
 */
public class HipUniformQuantizer extends Quantizer {
    public HipUniformQuantizer(int binNum) {
        super(binNum);
    }

    public HipUniformQuantizer() {
        super(Quantizer.DEFAULT_BIN_NUM);
    }

    @Override
    public void quantize(double[] values) {
        fill(HipCodec.encodeDenseUniformF64(HipCodec.ctx(), values, binNum));
    }

    @Override
    public void parallelQuantize(double[] values) {
        quantize(values);
    }

    private void fill(byte[] payload) {
        double[] info = HipCodec.info(payload);
        binNum = (int) info[0];
        n = (int) info[1];
        zeroIdx = (int) info[2];
        min = info[3];
        max = info[4];
        splits = new double[binNum - 1];
        System.arraycopy(info, 5, splits, 0, binNum - 1);
        bins = new int[n];
        HipCodec.getBins(payload, bins);
    }

    @Override
    public QuantizationType quantizationType() {
        return QuantizationType.UNIFORM;
    }
}
