from .mnist import main

raise SystemExit(main())
