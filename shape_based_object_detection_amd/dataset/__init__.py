"""Box codecs of the reference's ``dataset`` package (the I/O half is out of scope)."""
