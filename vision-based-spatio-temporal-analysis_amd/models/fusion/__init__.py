# fusion package
