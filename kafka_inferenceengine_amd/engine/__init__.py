"""Engine: device state, band descriptors and the LinearKalman driver."""
