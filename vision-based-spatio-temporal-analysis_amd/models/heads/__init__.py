# heads package
