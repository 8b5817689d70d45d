# encoders package
