"""Data formats: the device-resident Spectra (drop-in for pypulsar.formats)."""
